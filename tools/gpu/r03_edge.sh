# Varlen encode: edge units first with aligned partial stores, and the fused
# scan apply (passes 2+3 in one launch): parity, then A/B across builds and
# forms, then the tile-phase timeline.
set -e
timeout -k 10 400 python -u -m pytest tests/test_gpu_varlen.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/edge_tests.log 2>&1
timeout -k 10 300 python -u tools/lib_ab.py --op varlen --L 1472,ragged,512,1024 --libs fused=reliable-udp_amd/rudp/librudp.so,edge=reliable-udp_amd/build_ab/librudp_edge.so,head=reliable-udp_amd/build_ab/librudp_r03head.so > gpurun_out/edge_libab.json 2> gpurun_out/edge_libab.err
timeout -k 10 300 python -u tools/knob_ab.py --variants "btile:;ptile:51=0;bt2:51=2;bt2s16:51=2,59=23552;nofuse:60=0" --shapes varlen:1472,ragged > gpurun_out/edge_knob.json 2> gpurun_out/edge_knob.err
timeout -k 10 300 python -u tools/varlen_timeline.py > gpurun_out/edge_timeline.json 2> gpurun_out/edge_timeline.err
echo done
