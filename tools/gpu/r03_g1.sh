# round 3, call 1: GPU tests (all), C3 tile timeline (8 rotating sets, XCD order off/on), C3 trace + PMC
set -e
bash tools/gpu/run.sh tests
timeout -k 10 300 python -u tools/tile_timeline.py --L 64 --no-16m --sets 8 > gpurun_out/tl64.json 2> gpurun_out/tl64.err
timeout -k 10 300 python -u tools/tile_timeline.py --L 64 --no-16m --sets 8 --tune 5=1 > gpurun_out/tl64_xcd.json 2> gpurun_out/tl64_xcd.err
bash tools/gpu/run.sh trace c3_kt tools/run_kernel.py --op encode --L 64 --steps 50
bash tools/gpu/run.sh pmc c3 tools/run_kernel.py --op encode --L 64 --steps 20
bash tools/gpu/run.sh bench r03a
echo done
