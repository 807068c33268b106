# Varlen encode: the tile form chosen by the scan (pass 1 counts, pass 2
# decides) and one record per workgroup in the chosen form: parity, then A/B
# against the previous build and the forms.
set -e
timeout -k 10 400 python -u -m pytest tests/test_gpu_varlen.py tests/test_gpu_fuzz.py tests/test_gpu_c5.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/rec_tests.log 2>&1
timeout -k 10 300 python -u tools/lib_ab.py --op varlen --L 1472,ragged,1024,2048,4000 --libs rec=reliable-udp_amd/rudp/librudp.so,head=reliable-udp_amd/build_ab/librudp_r03head.so > gpurun_out/rec_libab.json 2> gpurun_out/rec_libab.err
timeout -k 10 300 python -u tools/knob_ab.py --variants "auto:;ptile:51=0;bt2:51=2;prec3:51=3" --shapes varlen:1472,ragged > gpurun_out/rec_knob.json 2> gpurun_out/rec_knob.err
echo done
