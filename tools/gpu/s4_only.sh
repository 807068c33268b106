# usage: bash tools/gpu/s4_only.sh MODE TAG [extra sweep args]
set -e
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
M=$1; T=$2; shift 2
timeout -k 10 300 python -u tools/sweep.py --only $M "$@" > $O/sweep_$T.json 2> $O/sweep_$T.err
echo done
