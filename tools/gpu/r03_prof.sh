# round 3: rocprofv3 kernel traces + FETCH_SIZE / WRITE_SIZE (separate passes) for every timed bench leg
set -e
R=tools/run_kernel.py
run() {  # tag, run_kernel args...
  tag=$1; shift
  bash tools/gpu/run.sh trace ${tag}_kt $R "$@"
  bash tools/gpu/run.sh pmc ${tag} $R "$@" --steps 10
}
run enc1472 --op encode --L 1472 --steps 30
run enc1024 --op encode --L 1024 --steps 30
run dec1472 --op decode --L 1472 --steps 30
run enc16M --op encode --L 1472 --n 16777216 --steps 6
run venc1472 --op encode_varlen --L 1472 --steps 30
run vdec1472 --op decode_varlen --L 1472 --steps 30
run vencrag --op encode_varlen --L 1472 --ragged --steps 30
run vdecrag --op decode_varlen --L 1472 --ragged --steps 30
run utf8 --op utf8 --L 1472 --steps 30
run dedup --op dedup --L 1 --steps 30
run venc1c --op encode_varlen --L 1 --layout rudp5 --steps 50
run vdec1c --op decode_varlen --L 1 --layout rudp5 --steps 50
echo done
