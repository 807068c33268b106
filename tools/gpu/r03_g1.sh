set -e
bash tools/gpu/run.sh tests -k "digests or reject_bad or config1 or receiver or c5_single" 
timeout -k 10 300 python -u tools/tile_timeline.py --L 64 --no-16m --sets 8 > gpurun_out/tl64.json 2> gpurun_out/tl64.err
timeout -k 10 300 python -u tools/tile_timeline.py --L 64 --no-16m --sets 8 --tune 5=1 > gpurun_out/tl64_xcd.json 2> gpurun_out/tl64_xcd.err
bash tools/gpu/run.sh trace c3_kt tools/run_kernel.py --op encode --L 64 --steps 50
bash tools/gpu/run.sh pmc c3 tools/run_kernel.py --op encode --L 64 --steps 20
echo done
