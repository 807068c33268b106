# small-frame decode frames per thread (tools build, knob 47), 1M x 1 B and 4 B, rudp5 with sideband checksums
set -e
for r in 1 2; do for v in 2 4 8; do for L in 1 4; do
  timeout -k 10 120 python -u tools/run_kernel.py --op decode_varlen --L $L --layout rudp5 --steps 400 --tune 47=$v >> gpurun_out/dfpt_ab.log 2>&1
done; done; done
echo done
