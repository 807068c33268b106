# One parameterised driver for the GPU box (run from the repo root under gpurun).
# Replaces the per-session scripts of round 1.  Every step has its own time
# limit; chain steps with && so a failure ends the call.
#
#   bash tools/gpu/run.sh tests [extra pytest args]        # pytest -m gpu
#   bash tools/gpu/run.sh smoke                            # __graft_entry__.smoke()
#   bash tools/gpu/run.sh bench TAG [bench.py args]        # one bench line -> gpurun_out/bench_TAG.json
#   bash tools/gpu/run.sh trace TAG PROG [args]            # rocprofv3 kernel trace + stats
#   bash tools/gpu/run.sh pmc TAG PROG [args]              # FETCH_SIZE and WRITE_SIZE, one pass each
#   bash tools/gpu/run.sh pmcsq TAG PROG [args]            # 8 SQ counters (wave cycles, waits, VALU/LDS) in one pass
#   bash tools/gpu/run.sh pmcvalu TAG PROG [args]          # VALU-busy view: 8 SQ + 2 GRBM counters in one pass
#   bash tools/gpu/run.sh sweep TAG [tools/sweep.py args]  # interleaved A/B sweep
#   bash tools/gpu/run.sh py TAG SCRIPT [args]             # any python tool, output to TAG.log
#
# PROG is a python script path (run as `python3 PROG`, directly after rocprofv3's --).
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
step=$1; shift
case "$step" in
  tests)
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread "$@" \
      > "$O/gpu_tests.log" 2>&1 ;;
  smoke)
    timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 ;;
  bench)
    tag=$1; shift
    timeout -k 10 600 python -u bench.py "$@" > "$O/bench_$tag.json" 2> "$O/bench_$tag.err" ;;
  trace)
    tag=$1; shift
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/$tag" -o run -- python3 "$@" \
      > "$O/$tag.log" 2>&1 ;;
  pmc)
    tag=$1; shift
    timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -f csv -d "$O/${tag}_fetch" -o run -- python3 "$@" \
      > "$O/${tag}_fetch.log" 2>&1
    timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -f csv -d "$O/${tag}_write" -o run -- python3 "$@" \
      > "$O/${tag}_write.log" 2>&1 ;;
  pmcsq)
    tag=$1; shift
    timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
      SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -f csv -d "$O/${tag}_sq" -o run \
      -- python3 "$@" > "$O/${tag}_sq.log" 2>&1 ;;
  pmcvalu)
    tag=$1; shift
    timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
      SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT -f csv -d "$O/${tag}_valu" -o run \
      -- python3 "$@" > "$O/${tag}_valu.log" 2>&1 ;;
  sweep)
    tag=$1; shift
    timeout -k 10 500 python -u tools/sweep.py "$@" > "$O/sweep_$tag.json" 2> "$O/sweep_$tag.err" ;;
  py)
    tag=$1; shift
    timeout -k 10 500 python -u "$@" > "$O/$tag.log" 2>&1 ;;
  *)
    echo "unknown step $step" >&2; exit 2 ;;
esac
echo "$step ok"
