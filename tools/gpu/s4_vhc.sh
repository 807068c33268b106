set -e
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_varlen.py -x -q --timeout 120 --timeout-method thread > $O/varlen_tests.log 2>&1
timeout -k 10 400 python -u tools/sweep.py --only opsknob --key 36 --values 0,1 --encode-L 1472,1024,256,64 --reps 15 > $O/sweep_vhc.json 2> $O/sweep_vhc.err
echo done
