set -e
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "decode" > $O/stage_tests.log 2>&1
timeout -k 10 400 python -u tools/sweep.py --only opsknob --key 34 --values 0,1 --encode-L 1472,256,64 --reps 15 > $O/sweep_stage.json 2> $O/sweep_stage.err
echo done
