# usage: bash tools/gpu/s4_knob.sh KEY VALUES LS TAG
set -e
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python -u tools/sweep.py --only knob --key $1 --values $2 --encode-L $3 --reps 15 > $O/sweep_$4.json 2> $O/sweep_$4.err
echo done
