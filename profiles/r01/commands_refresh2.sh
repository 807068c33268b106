# round-1 second refresh: full bench line, then rocprofv3 kernel traces + separate PMC passes
# (FETCH_SIZE, WRITE_SIZE) for encode (headline), decode-verify, copy-out decode, and kernel
# traces of the varlen encode/decode at 1M x 1472 B.  Summaries: tools/prof_summary.py.
set -e
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out
timeout -k 10 400 python bench.py > $R/gpurun_out/bench_r3.log 2>&1
P="timeout -k 10 240 rocprofv3"
$P --kernel-trace --stats -f csv -d $R/gpurun_out/p3_enc -o run -- python3 bench.py --no-legs --no-cpu-baseline > $R/gpurun_out/p3_enc.log 2>&1
$P --pmc FETCH_SIZE -f csv -d $R/gpurun_out/p3_enc_fetch -o run -- python3 bench.py --no-legs --no-cpu-baseline --steps 10 --warmup 2 > /dev/null 2>&1
$P --pmc WRITE_SIZE -f csv -d $R/gpurun_out/p3_enc_write -o run -- python3 bench.py --no-legs --no-cpu-baseline --steps 10 --warmup 2 > /dev/null 2>&1
for op in decode decode_copy; do
  $P --kernel-trace --stats -f csv -d $R/gpurun_out/p3_$op -o run -- python3 tools/run_kernel.py --op $op --steps 50 > $R/gpurun_out/p3_$op.log 2>&1
  $P --pmc FETCH_SIZE -f csv -d $R/gpurun_out/p3_${op}_fetch -o run -- python3 tools/run_kernel.py --op $op --steps 10 > /dev/null 2>&1
  $P --pmc WRITE_SIZE -f csv -d $R/gpurun_out/p3_${op}_write -o run -- python3 tools/run_kernel.py --op $op --steps 10 > /dev/null 2>&1
done
for op in encode_varlen decode_varlen; do
  $P --kernel-trace --stats -f csv -d $R/gpurun_out/p3_$op -o run -- python3 tools/run_kernel.py --op $op --L 1472 --steps 20 > $R/gpurun_out/p3_$op.log 2>&1
done
echo "refresh2 done"
