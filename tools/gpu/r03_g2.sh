# round 3, call 2: C3 small-tile tail sweep + timeline; varlen byte vs packet tiles (equal lengths) and ragged: traces + PMC
set -e
O=gpurun_out
timeout -k 10 400 python -u tools/tail_sweep.py --L 64 --reps 11 --percu=-1,5,7 > $O/tail64.json 2> $O/tail64.err
timeout -k 10 300 python -u tools/tile_timeline.py --L 64 --no-16m --sets 8 --tune 55=65536,56=32 > $O/tl64_tail.json 2> $O/tl64_tail.err
bash tools/gpu/run.sh trace vl_eq_pkt tools/run_kernel.py --op encode_varlen --tune 51=0 --steps 30
bash tools/gpu/run.sh trace vl_eq_bt tools/run_kernel.py --op encode_varlen --tune 51=2 --steps 30
bash tools/gpu/run.sh trace vl_eq_auto tools/run_kernel.py --op encode_varlen --steps 30
bash tools/gpu/run.sh trace vl_rag_auto tools/run_kernel.py --op encode_varlen --ragged --steps 30
bash tools/gpu/run.sh trace vl_rag_pkt tools/run_kernel.py --op encode_varlen --ragged --tune 51=0 --steps 30
bash tools/gpu/run.sh pmc vl_eq_pkt tools/run_kernel.py --op encode_varlen --tune 51=0 --steps 10
bash tools/gpu/run.sh pmc vl_eq_bt tools/run_kernel.py --op encode_varlen --tune 51=2 --steps 10
bash tools/gpu/run.sh pmc vl_rag_auto tools/run_kernel.py --op encode_varlen --ragged --steps 10
for t in vl_eq_pkt vl_eq_bt vl_rag_auto; do
  extra="--tune 51=0"; [ $t = vl_eq_bt ] && extra="--tune 51=2"; [ $t = vl_rag_auto ] && extra="--ragged"
  timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -f csv -d $O/${t}_wrreq -o run -- python3 tools/run_kernel.py --op encode_varlen $extra --steps 10 > $O/${t}_wrreq.log 2>&1
done
echo done
