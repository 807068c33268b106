set -e
timeout -k 10 400 python -u tools/knob_ab.py --variants "base:;t256:2=256;t256b512:2=256,10=512;t128b512:10=512;pc6:6=6;pc7:6=7" --shapes encode:64 --reps 11 > gpurun_out/ab64_geom.json 2> gpurun_out/ab64_geom.err
timeout -k 10 400 python -u tools/knob_ab.py --variants "base:;b512:10=512" --shapes encode:1472,encode:1024,encode:256 --reps 9 > gpurun_out/ab_b512.json 2> gpurun_out/ab_b512.err
echo done
