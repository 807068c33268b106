# round 3, call 3: persistent encode sweep (64 / 256 / 1024 / 1472 B), tail combos, varlen tile timelines
set -e
O=gpurun_out
timeout -k 10 300 python -u tools/tail_sweep.py --L 64 --reps 9 --persist=0,4,6,8 --tails=0,65536,98304 --tail-T=64 > $O/persist64.json 2> $O/persist64.err
timeout -k 10 300 python -u tools/tail_sweep.py --L 256 --reps 9 --persist=0,4,6,8 --tails=0 --sets 4 > $O/persist256.json 2> $O/persist256.err
timeout -k 10 300 python -u tools/tail_sweep.py --L 1472 --reps 9 --persist=0,3,4,5 --tails=0 --sets 1 > $O/persist1472.json 2> $O/persist1472.err
timeout -k 10 300 python -u tools/tail_sweep.py --L 1024 --reps 9 --persist=0,4,5 --tails=0 --sets 1 > $O/persist1024.json 2> $O/persist1024.err
timeout -k 10 300 python -u tools/varlen_timeline.py > $O/vtl.json 2> $O/vtl.err
echo done
