# Small-frame varlen decode: rudp5 sideband checksums prefetched with the tile's first offsets
set -e
timeout -k 10 400 python -u -m pytest tests/test_gpu_varlen.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/sdec_tests.log 2>&1
timeout -k 10 300 python -u tools/lib_ab.py --op vdecode --L 1,4,9,1472 --reps 15 --libs new=reliable-udp_amd/rudp/librudp.so,head=reliable-udp_amd/build_ab/librudp_rec.so > gpurun_out/sdec_libab.json 2> gpurun_out/sdec_libab.err
echo done
