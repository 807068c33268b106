# host-side HIP API costs of the small-frame varlen encode / decode calls (rocprofv3 --hip-trace --stats)
set -e
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --hip-trace --kernel-trace --stats -f csv -d gpurun_out/ht_venc1c -o run -- python3 tools/run_kernel.py --op encode_varlen --L 1 --layout rudp5 --steps 200 > gpurun_out/ht_venc1c.log 2>&1
timeout -k 10 200 rocprofv3 --hip-trace --kernel-trace --stats -f csv -d gpurun_out/ht_vdec1c -o run -- python3 tools/run_kernel.py --op decode_varlen --L 1 --layout rudp5 --steps 200 > gpurun_out/ht_vdec1c.log 2>&1
echo done
