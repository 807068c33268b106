# Session-4 refresh (LDS-DMA phase 1 default): GPU tests, full bench line, then
# rocprofv3 kernel trace + separate FETCH_SIZE / WRITE_SIZE passes of the
# headline encode (bench.py --no-legs).
set -e
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 400 python bench.py > $O/bench_s4r.log 2>&1
P="timeout -k 10 240 rocprofv3"
$P --kernel-trace --stats -f csv -d $O/p5_enc -o run -- python3 bench.py --no-legs --no-cpu-baseline > $O/p5_enc.log 2>&1
$P --pmc FETCH_SIZE -f csv -d $O/p5_enc_fetch -o run -- python3 bench.py --no-legs --no-cpu-baseline --steps 10 --warmup 2 > /dev/null 2>&1
$P --pmc WRITE_SIZE -f csv -d $O/p5_enc_write -o run -- python3 bench.py --no-legs --no-cpu-baseline --steps 10 --warmup 2 > /dev/null 2>&1
echo "refresh done"
