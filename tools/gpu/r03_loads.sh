# Which of a byte tile's first loads costs: the form counter or the packet form's offsets
set -e
timeout -k 10 300 python -u tools/knob_ab.py --variants "ptile:51=0;bt2:51=2;bt2nol:51=2,61=4;bt2noover:51=2,61=16;bt2nopfo:51=2,61=32" --shapes varlen:1472,ragged --reps 11 > gpurun_out/loads_knob.json 2> gpurun_out/loads_knob.err
echo done
