# round 3 refresh: rocprofv3 kernel trace (per-dispatch durations) + FETCH_SIZE /
# WRITE_SIZE (separate passes) for every timed bench leg, each run warmed for
# 30 ms before its timed launches (tools/run_kernel.py).  Summaries are made
# in the build container by tools/r03_summaries.py.
set -e
R=tools/run_kernel.py
run() {  # tag, run_kernel args...
  tag=$1; shift
  bash tools/gpu/run.sh trace p2_${tag}_kt $R "$@"
  bash tools/gpu/run.sh pmc p2_${tag} $R "$@" --steps 10
}
run enc1472 --op encode --L 1472 --steps 40
run enc1024 --op encode --L 1024 --steps 40
run enc64 --op encode --L 64 --steps 80
run dec1472 --op decode --L 1472 --steps 40
run enc16M --op encode --L 1472 --n 16777216 --steps 8
run venc1472 --op encode_varlen --L 1472 --steps 40
run vdec1472 --op decode_varlen --L 1472 --steps 40
run vencrag --op encode_varlen --L 1472 --ragged --steps 40
run vdecrag --op decode_varlen --L 1472 --ragged --steps 40
run utf8 --op utf8 --L 1472 --steps 40
run dedup --op dedup --L 1 --steps 60
run venc1c --op encode_varlen --L 1 --layout rudp5 --steps 80
run vdec1c --op decode_varlen --L 1 --layout rudp5 --steps 80
echo done
