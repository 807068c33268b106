# Packet tiles through records vs from frame_off at equal lengths: the grid's
# empty workgroups (spans = packet tiles with S = 16 x 1472) and the LDS slots
set -e
timeout -k 10 300 python -u tools/knob_ab.py --variants "ptile:51=0;prec3:51=3;prec3_s16:51=3,59=23552;prec3_slot16:51=3,61=2;prec3_both:51=3,59=23552,61=2;auto:" --shapes varlen:1472,varlen:1024 --reps 11 > gpurun_out/prec_knob.json 2> gpurun_out/prec_knob.err
echo done
