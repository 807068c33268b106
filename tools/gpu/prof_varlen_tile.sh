# varlen encode through LDS tiles: parity tests, tile-vs-vector sweep, and
# rocprofv3 kernel traces + FETCH/WRITE passes of the MTU-size varlen encode.
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_varlen.py -x -q --timeout 120 --timeout-method thread > $O/varlen_tests.log 2>&1
timeout -k 10 200 python tools/sweep.py --only varlen_enc --reps 9 > $O/sweep_varlen_enc.json 2> $O/sweep_varlen_enc.err
P="timeout -k 10 240 rocprofv3"
for L in 1472 64; do
  $P --kernel-trace --stats -f csv -d $O/pv_enc_$L -o run -- python3 tools/run_kernel.py --op encode_varlen --L $L --steps 20 > $O/pv_enc_$L.log 2>&1
done
$P --pmc FETCH_SIZE -f csv -d $O/pv_enc_fetch -o run -- python3 tools/run_kernel.py --op encode_varlen --L 1472 --steps 10 > /dev/null 2>&1
$P --pmc WRITE_SIZE -f csv -d $O/pv_enc_write -o run -- python3 tools/run_kernel.py --op encode_varlen --L 1472 --steps 10 > /dev/null 2>&1
echo done
