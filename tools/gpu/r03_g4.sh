# round 3, call 4: varlen tile kernel (block sums in their own LDS, map in the sum pass, two-lane header
# chunks, per-chunk fast phase 2): varlen GPU tests, phase timeline, bench varlen legs
set -e
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_varlen.py tests/test_gpu_fuzz.py -x -q --timeout 180 --timeout-method thread > $O/vt_tests.log 2>&1
timeout -k 10 300 python -u tools/varlen_timeline.py > $O/vtl3.json 2> $O/vtl3.err
bash tools/gpu/run.sh bench r03c --no-cpu-baseline
echo done
