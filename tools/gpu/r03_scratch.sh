# Per-thread stream scratch instead of a pool alloc/free per call: all GPU tests, then A/B
set -e
bash tools/gpu/run.sh tests
timeout -k 10 300 python -u tools/lib_ab.py --op varlen --L 1,4,1472,ragged --reps 15 --libs new=reliable-udp_amd/rudp/librudp.so,prev=reliable-udp_amd/build_ab/librudp_small1.so > gpurun_out/scratch_libab.json 2> gpurun_out/scratch_libab.err
timeout -k 10 200 python -u tools/alloc_probe.py > gpurun_out/scratch_alloc_probe.json 2> gpurun_out/scratch_alloc_probe.err
echo done
