# usage: bash tools/gpu/s4_multi.sh TAG LS "SPECS" [REPS]
set -e
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 400 python -u tools/sweep.py --only multi --encode-L $2 --specs "$3" --reps ${4:-15} > $O/sweep_$1.json 2> $O/sweep_$1.err
echo done
