set -e
timeout -k 10 400 python -u tools/knob_ab.py --variants "base:;noscr:37=0;b128:10=128;b128_noscr:10=128,37=0" --shapes encode:64,encode:256 --reps 11 > gpurun_out/ab64_b128.json 2> gpurun_out/ab64_b128.err
echo done
