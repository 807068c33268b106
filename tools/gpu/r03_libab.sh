set -e
timeout -k 10 300 python -u tools/lib_ab.py --libs product=reliable-udp_amd/rudp/librudp.so,tools=reliable-udp_amd/rudp/librudp_tools.so,r02=reliable-udp_amd/build_ab/librudp_r02.so > gpurun_out/lib_ab.json 2> gpurun_out/lib_ab.err
echo done
