# Varlen encode: byte tiles always over spans of tile_T x hint (no per-call
# choice, no packet-form loads): parity, then A/B against the previous build and forms.
set -e
timeout -k 10 400 python -u -m pytest tests/test_gpu_varlen.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/force_tests.log 2>&1
timeout -k 10 300 python -u tools/lib_ab.py --op varlen --L 1472,ragged,1024,2048,4000 --libs force=reliable-udp_amd/rudp/librudp.so,head=reliable-udp_amd/build_ab/librudp_r03head.so > gpurun_out/force_libab.json 2> gpurun_out/force_libab.err
timeout -k 10 300 python -u tools/knob_ab.py --variants "bt1:;ptile:51=0;bt2:51=2;auto3:51=3" --shapes varlen:1472,ragged,varlen:1024 > gpurun_out/force_knob.json 2> gpurun_out/force_knob.err
echo done
