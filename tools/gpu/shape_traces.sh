# Kernel traces of the checked varlen encode on a few shapes, two builds.
set -e
B=$PWD/reliable-udp_amd/rudp/librudp_base.so
RUDP_LIB=$B bash tools/gpu/run.sh trace sh_base tools/varlen_shapes.py --only L64,L512,U0-512 --reps 20
bash tools/gpu/run.sh trace sh_new tools/varlen_shapes.py --only L64,L512,U0-512 --reps 20
