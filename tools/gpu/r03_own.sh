# Varlen encode: edge chunks owned whole by one tile (edge_owned), the owned
# head chunk prebuilt by frame 0's leaders: parity, then A/B across builds and forms.
set -e
timeout -k 10 400 python -u -m pytest tests/test_gpu_varlen.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/own_tests.log 2>&1
timeout -k 10 300 python -u tools/lib_ab.py --op varlen --L 1472,ragged,1024,512 --libs own4=reliable-udp_amd/rudp/librudp.so,head=reliable-udp_amd/build_ab/librudp_r03head.so > gpurun_out/own_libab.json 2> gpurun_out/own_libab.err
timeout -k 10 300 python -u tools/knob_ab.py --variants "btile:;ptile:51=0;bt2:51=2;bt2noedge:51=2,61=1;bt2nol:51=2,61=4" --shapes varlen:1472,ragged > gpurun_out/own_knob.json 2> gpurun_out/own_knob.err
echo done
