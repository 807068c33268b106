set -e
L=product=reliable-udp_amd/rudp/librudp.so,tools=reliable-udp_amd/rudp/librudp_tools.so,r02=reliable-udp_amd/build_ab/librudp_r02.so
timeout -k 10 300 python -u tools/lib_ab.py --op decode --L 1472,1024,256 --libs $L > gpurun_out/lib_ab_dec.json 2> gpurun_out/lib_ab_dec.err
echo done
