# round-1 profile refresh: encode (headline), decode-verify and copy-out decode, 1M x 1472 B rudp7
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/p2_enc -o run -- python3 bench.py --no-legs --no-cpu-baseline > gpurun_out/p2_enc.log 2>&1 && \
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -f csv -d $R/gpurun_out/p2_enc_fetch -o run -- python3 bench.py --no-legs --no-cpu-baseline --steps 10 --warmup 2 > /dev/null 2>&1 && \
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -f csv -d $R/gpurun_out/p2_enc_write -o run -- python3 bench.py --no-legs --no-cpu-baseline --steps 10 --warmup 2 > /dev/null 2>&1 && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/p2_dec -o run -- python3 tools/run_kernel.py --op decode --steps 50 > gpurun_out/p2_dec.log 2>&1 && \
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -f csv -d $R/gpurun_out/p2_dec_fetch -o run -- python3 tools/run_kernel.py --op decode --steps 10 > /dev/null 2>&1 && \
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -f csv -d $R/gpurun_out/p2_dec_write -o run -- python3 tools/run_kernel.py --op decode --steps 10 > /dev/null 2>&1 && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/p2_cpy -o run -- python3 tools/run_kernel.py --op decode_copy --steps 50 > gpurun_out/p2_cpy.log 2>&1 && \
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -f csv -d $R/gpurun_out/p2_cpy_fetch -o run -- python3 tools/run_kernel.py --op decode_copy --steps 10 > /dev/null 2>&1 && \
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -f csv -d $R/gpurun_out/p2_cpy_write -o run -- python3 tools/run_kernel.py --op decode_copy --steps 10 > /dev/null 2>&1
echo "prof rc=$?"
