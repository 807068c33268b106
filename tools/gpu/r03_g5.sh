# round 3, call 5: transport GPU tests (batched relay), SQ counters of the varlen and fixed encode tiles, bench
set -e
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_transport.py -x -q -m gpu --timeout 120 --timeout-method thread > $O/tr_tests.log 2>&1
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $C -f csv -d $O/sq_venc -o run -- python3 tools/run_kernel.py --op encode_varlen --steps 10 > $O/sq_venc.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc $C -f csv -d $O/sq_enc -o run -- python3 tools/run_kernel.py --op encode --steps 10 > $O/sq_enc.log 2>&1
bash tools/gpu/run.sh bench r03d --no-cpu-baseline
echo done
