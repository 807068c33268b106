# Kernel traces: 1M x 1472 B equal lengths, automatic tile form vs packet tiles.
set -e
R=tools/run_kernel.py
bash tools/gpu/run.sh trace eq_auto $R --op encode_varlen --steps 20
bash tools/gpu/run.sh trace eq_packet $R --op encode_varlen --steps 20 --tune 51=0
