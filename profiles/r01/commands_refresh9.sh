# Session-4 refresh 6 (64-B dealing for every encode tile, decode copy-out cap,
# varlen tile size and budgets, packed UTF-8 tiles): tests, smoke, bench, traces + PMC,
# C3 (1M x 64 B) encode kernel trace + PMC.
set -e
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python bench.py > $O/bench_s4r7.log 2>&1
P="timeout -k 10 240 rocprofv3"
$P --kernel-trace --stats -f csv -d $O/p12_enc -o run -- python3 bench.py --no-legs --no-cpu-baseline > $O/p12_enc.log 2>&1
$P --pmc FETCH_SIZE -f csv -d $O/p12_enc_fetch -o run -- python3 bench.py --no-legs --no-cpu-baseline --steps 10 --warmup 2 > /dev/null 2>&1
$P --pmc WRITE_SIZE -f csv -d $O/p12_enc_write -o run -- python3 bench.py --no-legs --no-cpu-baseline --steps 10 --warmup 2 > /dev/null 2>&1
$P --kernel-trace --stats -f csv -d $O/p12_c3 -o run -- python3 tools/run_kernel.py --op encode --L 64 --steps 50 > $O/p12_c3.log 2>&1
$P --pmc FETCH_SIZE -f csv -d $O/p12_c3_fetch -o run -- python3 tools/run_kernel.py --op encode --L 64 --steps 10 > /dev/null 2>&1
$P --pmc WRITE_SIZE -f csv -d $O/p12_c3_write -o run -- python3 tools/run_kernel.py --op encode --L 64 --steps 10 > /dev/null 2>&1
echo "refresh6 done"
