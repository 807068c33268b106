set -e
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 400 python -u tools/sweep.py --only opsknob --key 30 --values=-1,0 --encode-L 1472,1024,256,64 --reps 15 > $O/sweep_early.json 2> $O/sweep_early.err
echo done
