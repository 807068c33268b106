set -e
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_span.py -x -q --timeout 120 --timeout-method thread > $O/span_tests.log 2>&1
timeout -k 10 400 python -u tools/sweep.py --only multi --encode-L 64,256,1472 --specs "funnel:37=0;scratch:37=1" --reps 21 > $O/sweep_scr.json 2> $O/sweep_scr.err
echo done
