# round 3, call 6: LDS windows from aligned b128 pairs (knob 58) A/B; SQ bank conflicts with it on
set -e
O=gpurun_out
timeout -k 10 400 python -u tools/knob_ab.py --knob 58 --values 0,1 --shapes encode:1472,encode:1024,encode:64,varlen:1472,ragged > $O/ab_win128.json 2> $O/ab_win128.err
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $C -f csv -d $O/sq_venc128 -o run -- python3 tools/run_kernel.py --op encode_varlen --steps 10 --tune 58=1 > $O/sq_venc128.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc $C -f csv -d $O/sq_enc128 -o run -- python3 tools/run_kernel.py --op encode --steps 10 --tune 58=1 > $O/sq_enc128.log 2>&1
echo done
