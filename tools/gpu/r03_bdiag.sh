# Why byte tiles lose at equal lengths: tile-phase timelines and A/B of
# ablations (span bytes = 16 packets, LDS slots, packet-form loads, edge units).
set -e
F="ptile:51=0;bt2:51=2;bt2s16:51=2,59=23552;bt2s16slot:51=2,59=23552,61=2;bt2s16nol:51=2,59=23552,61=4;bt2noedge:51=2,61=1"
timeout -k 10 300 python -u tools/knob_ab.py --variants "$F" --shapes varlen:1472 > gpurun_out/bdiag_knob.json 2> gpurun_out/bdiag_knob.err
timeout -k 10 400 python -u tools/varlen_timeline.py --shapes equal_1472 --forms "$F" > gpurun_out/bdiag_timeline.json 2> gpurun_out/bdiag_timeline.err
echo done
