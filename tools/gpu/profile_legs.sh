# rocprofv3 kernel trace (per-dispatch durations) + FETCH_SIZE / WRITE_SIZE
# (separate passes) for every timed bench leg, each run warmed for 30 ms
# before its timed launches (tools/run_kernel.py).  Outputs gpurun_out/<P>_<leg>*;
# tools/leg_summaries.py --prefix <P> --round <round> turns them into profiles/.
#   bash tools/gpu/profile_legs.sh PREFIX [leg ...]    (no legs: all of them)
set -e
P=$1; shift
R=tools/run_kernel.py
declare -A LEG=(
  [enc1472]="--op encode --L 1472 --steps 40"
  [enc1024]="--op encode --L 1024 --steps 40"
  [enc64]="--op encode --L 64 --steps 80"
  [dec1472]="--op decode --L 1472 --steps 40"
  [decu8_1472]="--op decode --utf8 --L 1472 --steps 40"
  [decu8text]="--op decode --utf8 --text --L 1472 --steps 40"
  [enc16M]="--op encode --L 1472 --n 16777216 --steps 8"
  [venc1472]="--op encode_varlen --L 1472 --steps 40"
  [vdec1472]="--op decode_varlen --L 1472 --steps 40"
  [vdecu8_1472]="--op decode_varlen --utf8 --L 1472 --steps 40"
  [vencrag]="--op encode_varlen --L 1472 --ragged --steps 40"
  [vdecrag]="--op decode_varlen --L 1472 --ragged --steps 40"
  [vdecu8rag]="--op decode_varlen --utf8 --L 1472 --ragged --steps 40"
  [utf8]="--op utf8 --L 1472 --steps 40"
  [dedup]="--op dedup --L 1 --steps 60"
  [venc1c]="--op encode_varlen --L 1 --layout rudp5 --steps 80"
  [vdec1c]="--op decode_varlen --L 1 --layout rudp5 --steps 80"
  [vdecu8_1c]="--op decode_varlen --utf8 --L 1 --layout rudp5 --steps 80"
  [senc1c]="--op encode --L 1 --layout rudp5 --steps 80"
  [sdecu8_1c]="--op decode --utf8 --L 1 --layout rudp5 --steps 80"
  [senc1000]="--op encode --L 1000 --steps 40"
)
legs=("$@")
[ ${#legs[@]} -eq 0 ] && legs=(enc1472 enc1024 enc64 dec1472 decu8_1472 decu8text enc16M venc1472 vdec1472 vdecu8_1472 \
                               vencrag vdecrag vdecu8rag utf8 dedup venc1c vdec1c vdecu8_1c senc1c sdecu8_1c senc1000)
for leg in "${legs[@]}"; do
  bash tools/gpu/run.sh trace ${P}_${leg}_kt $R ${LEG[$leg]}
  bash tools/gpu/run.sh pmc ${P}_${leg} $R ${LEG[$leg]} --steps 10
done
echo profile_legs ok
