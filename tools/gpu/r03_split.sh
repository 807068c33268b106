# Sub-tile split of overflowing varlen tiles: parity, then A/B against the
# previous build and packet tiles vs byte tiles.
set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_varlen.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/split_tests.log 2>&1
timeout -k 10 300 python -u tools/lib_ab.py --op varlen --L 1472,1024,512,ragged --libs new=reliable-udp_amd/rudp/librudp.so,head=reliable-udp_amd/build_ab/librudp_r03head.so > gpurun_out/split_libab.json 2> gpurun_out/split_libab.err
timeout -k 10 300 python -u tools/knob_ab.py --variants "btile:;ptile:51=0;ptile125:51=0,39=125;ptile100:51=0,39=100" --shapes ragged,varlen:1472 > gpurun_out/split_knob.json 2> gpurun_out/split_knob.err
echo done
