export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --share-device --steps 10 --warmup 2 > gpurun_out/bench_n2_shared.log 2>&1; echo "n2 rc=$?"; tail -1 gpurun_out/bench_n2_shared.log | cut -c1-400
timeout -k 10 300 python bench.py > gpurun_out/bench_full2.log 2>&1; echo "bench rc=$?"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_enc -o run -- python3 bench.py --no-legs --no-cpu-baseline > gpurun_out/prof_enc.log 2>&1 && \
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -f csv -d $R/gpurun_out/prof_enc_fetch -o run -- python3 bench.py --no-legs --no-cpu-baseline --steps 10 --warmup 2 > /dev/null 2>&1 && \
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -f csv -d $R/gpurun_out/prof_enc_write -o run -- python3 bench.py --no-legs --no-cpu-baseline --steps 10 --warmup 2 > /dev/null 2>&1 && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_dec -o run -- python3 tools/run_kernel.py --op decode --steps 50 > gpurun_out/prof_dec.log 2>&1 && \
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -f csv -d $R/gpurun_out/prof_dec_fetch -o run -- python3 tools/run_kernel.py --op decode --steps 10 > /dev/null 2>&1 && \
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -f csv -d $R/gpurun_out/prof_dec_write -o run -- python3 tools/run_kernel.py --op decode --steps 10 > /dev/null 2>&1
echo "prof rc=$?"
