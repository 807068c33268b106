set -e
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 python -u tools/sweep.py --only multi --encode-L 64 --specs "t0:2=0;t64:2=64;t256:2=256;t32:2=32" --reps 21 > $O/sweep_t64.json 2> $O/sweep_t64.err
timeout -k 10 300 python -u tools/sweep.py --only multi --encode-L 256,512 --specs "t0:2=0;t16:2=16;t64:2=64;t128:2=128" --reps 15 > $O/sweep_t256.json 2> $O/sweep_t256.err
echo done
