# Session-5 refresh 3 (varlen decode/UTF-8 tiles sized by bytes, from 128-B hints) (varlen early frame offsets + coded chunk map): GPU tests,
# smoke, bench, headline encode trace + PMC, varlen encode/decode traces + PMC.
set -e
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python bench.py > $O/bench_s5r3.log 2>&1
P="timeout -k 10 240 rocprofv3"
$P --kernel-trace --stats -f csv -d $O/p15_enc -o run -- python3 bench.py --no-legs --no-cpu-baseline > $O/p15_enc.log 2>&1
$P --pmc FETCH_SIZE -f csv -d $O/p15_enc_fetch -o run -- python3 bench.py --no-legs --no-cpu-baseline --steps 10 --warmup 2 > /dev/null 2>&1
$P --pmc WRITE_SIZE -f csv -d $O/p15_enc_write -o run -- python3 bench.py --no-legs --no-cpu-baseline --steps 10 --warmup 2 > /dev/null 2>&1
for op in encode_varlen decode_varlen; do
  $P --kernel-trace --stats -f csv -d $O/pv7_$op -o run -- python3 tools/run_kernel.py --op $op --steps 40 > $O/pv7_$op.log 2>&1
  $P --pmc FETCH_SIZE -f csv -d $O/pv7_${op}_fetch -o run -- python3 tools/run_kernel.py --op $op --steps 10 > /dev/null 2>&1
  $P --pmc WRITE_SIZE -f csv -d $O/pv7_${op}_write -o run -- python3 tools/run_kernel.py --op $op --steps 10 > /dev/null 2>&1
done
echo "s5 refresh done"
