# Dedup in one launch for short frames (the table pass hashes its own frames): parity, then A/B (tools build, knob 62)
set -e
timeout -k 10 400 python -u -m pytest tests/ -m gpu -x -q -k "dedup or retrans or relay or transport" --timeout 120 --timeout-method thread > gpurun_out/dedup_tests.log 2>&1
for v in 0 1 0 1; do timeout -k 10 120 python -u tools/run_kernel.py --op dedup --L 1 --steps 400 --tune 62=$v >> gpurun_out/dedup_ab.log 2>&1; done
echo done
