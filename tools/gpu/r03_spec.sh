# Small-frame varlen encode: speculative payload-run load at the hinted base
set -e
timeout -k 10 400 python -u -m pytest tests/test_gpu_varlen.py tests/test_gpu_fuzz.py tests/test_transport.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/spec_tests.log 2>&1
timeout -k 10 300 python -u tools/lib_ab.py --op varlen --L 1,4,9,15 --reps 15 --libs new=reliable-udp_amd/rudp/librudp.so,prev=reliable-udp_amd/build_ab/librudp_small1.so > gpurun_out/spec_libab.json 2> gpurun_out/spec_libab.err
echo done
