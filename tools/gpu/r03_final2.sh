# round 3, final tree: all GPU tests, smoke, bench, and the small-frame encode re-profiled
set -e
bash tools/gpu/run.sh tests
bash tools/gpu/run.sh smoke
bash tools/gpu/run.sh bench r03i
R=tools/run_kernel.py
bash tools/gpu/run.sh trace p2_venc1c_kt $R --op encode_varlen --L 1 --layout rudp5 --steps 80
bash tools/gpu/run.sh pmc p2_venc1c $R --op encode_varlen --L 1 --layout rudp5 --steps 10
echo done
