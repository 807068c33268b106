# rocprofv3 kernel-trace of the varlen encode/decode at MTU size (tools/run_kernel.py)
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for op in encode_varlen decode_varlen; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/prof_$op -o run -- \
    python3 tools/run_kernel.py --op $op --L 1472 --steps 10 > $R/gpurun_out/prof_$op.log 2>&1
done
