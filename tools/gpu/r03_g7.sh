# round 3, call 7: dedup changes (tests + trace + PMC), transport tests, bench
set -e
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_varlen.py tests/test_transport.py -x -q -m gpu --timeout 180 --timeout-method thread > $O/g7_tests.log 2>&1
bash tools/gpu/run.sh trace dedup2_kt tools/run_kernel.py --op dedup --L 1 --steps 30
bash tools/gpu/run.sh pmc dedup2 tools/run_kernel.py --op dedup --L 1 --steps 10
bash tools/gpu/run.sh bench r03e --no-cpu-baseline
echo done
