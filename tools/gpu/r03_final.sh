# round 3: all GPU tests, smoke, bench, and the varlen encode legs re-profiled
# after the scan-chosen tile records (same steps as tools/gpu/r03_prof2.sh)
set -e
bash tools/gpu/run.sh tests
bash tools/gpu/run.sh smoke
bash tools/gpu/run.sh bench r03h
R=tools/run_kernel.py
run() {
  tag=$1; shift
  bash tools/gpu/run.sh trace p2_${tag}_kt $R "$@"
  bash tools/gpu/run.sh pmc p2_${tag} $R "$@" --steps 10
}
run venc1472 --op encode_varlen --L 1472 --steps 40
run vencrag --op encode_varlen --L 1472 --ragged --steps 40
echo done
