set -e
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
#timeout -k 10 300 python -u -m pytest tests/test_gpu_span.py -x -q --timeout 120 --timeout-method thread > $O/span_tests.log 2>&1
#timeout -k 10 300 python -u tools/sweep.py --only knob --key 26 --values 0,1 --encode-L 1472,1024,256 --reps 15 > $O/sweep_span.json 2> $O/sweep_span.err
#timeout -k 10 300 python -u tools/sweep.py --only knob --key 27 --values 8192,4096,12288,16384 --pre 26=1 --encode-L 1472 --reps 11 > $O/sweep_spanS.json 2> $O/sweep_spanS.err
timeout -k 10 300 python -u tools/sweep.py --only knob --key 27 --values 8192,12288,16384,24576 --pre 26=1,6=0 --encode-L 1472,1024 --reps 11 > $O/sweep_spanP.json 2> $O/sweep_spanP.err
echo done
