set -e
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python -u tools/sweep.py --only encode --encode-L 1472,1024 --blocks 256 --tiles 8,16 --percu 0,3,4,5,6,8 --reps 11 > $O/sweep_percu.json 2> $O/sweep_percu.err
echo done
