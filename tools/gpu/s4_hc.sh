set -e
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_span.py -x -q --timeout 120 --timeout-method thread > $O/span_tests.log 2>&1
timeout -k 10 400 python -u tools/sweep.py --only multi --encode-L 1472,1024,256,64 --specs "tile:29=0,30=0;hc:29=1,30=0;hce:29=1,30=1;early:29=0,30=1" --reps 21 > $O/sweep_hc.json 2> $O/sweep_hc.err
echo done
