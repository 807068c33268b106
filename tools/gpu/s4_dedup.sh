set -e
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_varlen.py -x -q --timeout 120 --timeout-method thread -k dedup > $O/dedup_tests.log 2>&1
timeout -k 10 300 python -u tools/dedup_sweep.py > $O/dedup_sweep.json 2> $O/dedup_sweep.err
echo done
