# kernel traces: packet tiles from frame_off (51=0) vs through records (51=3), equal 1472-B lengths
set -e
bash tools/gpu/run.sh trace prec_p0 tools/run_kernel.py --op encode_varlen --L 1472 --steps 40 --tune 51=0
bash tools/gpu/run.sh trace prec_p3 tools/run_kernel.py --op encode_varlen --L 1472 --steps 40 --tune 51=3
echo done
