# Session-4: current varlen encode/decode (1M x 1472, packed, rudp7) kernel traces + PMC traffic.
set -e
export TMPDIR=/tmp; R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
P="timeout -k 10 240 rocprofv3"
for op in encode_varlen decode_varlen; do
  $P --kernel-trace --stats -f csv -d $O/pv_$op -o run -- python3 tools/run_kernel.py --op $op --steps 40 > $O/pv_$op.log 2>&1
  $P --pmc FETCH_SIZE -f csv -d $O/pv_${op}_fetch -o run -- python3 tools/run_kernel.py --op $op --steps 10 > /dev/null 2>&1
  $P --pmc WRITE_SIZE -f csv -d $O/pv_${op}_write -o run -- python3 tools/run_kernel.py --op $op --steps 10 > /dev/null 2>&1
done
echo "varlen prof done"
