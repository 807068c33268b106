# round 3, final tree after the per-thread scratch: smoke, bench, small-frame encode and dedup re-profiled
set -e
bash tools/gpu/run.sh smoke
bash tools/gpu/run.sh bench r03j
R=tools/run_kernel.py
run() {
  tag=$1; shift
  bash tools/gpu/run.sh trace p2_${tag}_kt $R "$@"
  bash tools/gpu/run.sh pmc p2_${tag} $R "$@" --steps 10
}
run venc1c --op encode_varlen --L 1 --layout rudp5 --steps 80
run dedup --op dedup --L 1 --steps 60
echo done
