set -e
R=tools/run_kernel.py
bash tools/gpu/run.sh trace bt_eq_off $R --op encode_varlen --steps 20
bash tools/gpu/run.sh trace bt_eq_on $R --op encode_varlen --steps 20 --tune 51=1,52=2
bash tools/gpu/run.sh trace bt_rg_off $R --op encode_varlen --steps 20 --ragged
bash tools/gpu/run.sh trace bt_rg_on $R --op encode_varlen --steps 20 --ragged --tune 51=1,52=2
