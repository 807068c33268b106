# Round-6 profiles (from the repo root, under gpurun), then on the build host:
#   python3 tools/leg_summaries.py --prefix p6a --round r06 <legs>; ... --prefix p6b ...
bash tools/gpu/profile_legs.sh p6a enc1472 enc1024 enc64 dec1472 decu8_1472 decu8text enc16M venc1472 vdec1472 vdecu8_1472
bash tools/gpu/profile_legs.sh p6b vencrag vdecrag vdecu8rag utf8 dedup venc1c vdec1c vdecu8_1c senc1c sdecu8_1c senc1000
bash tools/gpu/run.sh pmcsq p6text tools/run_kernel.py --op decode --utf8 --text --L 1472 --steps 10
bash tools/gpu/run.sh pmcvalu p6text tools/run_kernel.py --op decode --utf8 --text --L 1472 --steps 60
bash tools/gpu/run.sh pmcsq p6ascii tools/run_kernel.py --op decode --utf8 --L 1472 --steps 10
bash tools/gpu/run.sh bench r06c
# python3 tools/clock_spread.py gpurun_out/p6text_valu/run_counter_collection.csv --kernel decode_tile_kernel \
#   --json profiles/r06/utf8_text_clock_spread.json
# after the last UTF-8 kernel changes:
bash tools/gpu/profile_legs.sh p6c decu8_1472 decu8text vdecu8_1472 vdecu8rag utf8
bash tools/gpu/run.sh pmcsq p6ctext tools/run_kernel.py --op decode --utf8 --text --L 1472 --steps 10
bash tools/gpu/run.sh pmcvalu p6ctext tools/run_kernel.py --op decode --utf8 --text --L 1472 --steps 60
bash tools/gpu/run.sh bench r06e
# host zero-copy A/Bs (old library via RUDP_LIB, alternating processes):
#   python -u tools/e2e_varlen_leg.py --reps 9   -> profiles/r06/sweeps/host_zero_copy_*_ab.json
# round end on the final tree:
bash tools/gpu/run.sh tests && bash tools/gpu/run.sh smoke && bash tools/gpu/run.sh bench r06g
