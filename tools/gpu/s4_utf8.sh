set -e
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_varlen.py -x -q --timeout 120 --timeout-method thread > $O/utf8_tests.log 2>&1
timeout -k 10 400 python -u tools/sweep.py --only utf8 --reps 15 > $O/sweep_utf8.json 2> $O/sweep_utf8.err
echo done
