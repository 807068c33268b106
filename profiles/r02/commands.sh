# Round 2 GPU commands (each run as `gpurun -- '<line>'`; tools/gpu/run.sh wraps every
# step in its own time limit and writes under gpurun_out/).
bash tools/gpu/run.sh tests                                     # pytest -m gpu
bash tools/gpu/run.sh bench r02f                                # bench_r02f.json
# headline encode trace + PMC (bench.py's own command; rocprof avg vs bench events)
bash tools/gpu/run.sh trace enc1M bench.py --no-legs --no-cpu-baseline
bash tools/gpu/run.sh pmc enc1M bench.py --no-legs --no-cpu-baseline --steps 10 --warmup 2
bash tools/gpu/run.sh trace dec1M tools/run_kernel.py --op decode --steps 50
bash tools/gpu/run.sh pmc dec1M tools/run_kernel.py --op decode --steps 10
bash tools/gpu/run.sh trace vdec1472 tools/run_kernel.py --op decode_varlen --steps 40
bash tools/gpu/run.sh pmc vdec1472 tools/run_kernel.py --op decode_varlen --steps 10
bash tools/gpu/run.sh trace enc16M tools/run_kernel.py --op encode --n 16777216 --steps 20
bash tools/gpu/run.sh pmc enc16M tools/run_kernel.py --op encode --n 16777216 --steps 5
bash tools/gpu/run.sh trace venc1 tools/run_kernel.py --op encode_varlen --L 1 --steps 40
bash tools/gpu/run.sh trace vdec1 tools/run_kernel.py --op decode_varlen --L 1 --steps 40
# UTCL1 translation counters, 16M vs 1M encode (one pass each: 4 TCP counters)
timeout -s KILL 200 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_MULTI_MISS_sum -f csv -d gpurun_out/tlb/m16 -o run -- python3 tools/run_kernel.py --op encode --n 16777216 --steps 4
timeout -s KILL 200 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_MULTI_MISS_sum -f csv -d gpurun_out/tlb/m1 -o run -- python3 tools/run_kernel.py --op encode --steps 8
# sweeps (profiles/r02/sweeps/)
bash tools/gpu/run.sh py cache_res2 tools/cache_residency.py      # cache_residency.json
bash tools/gpu/run.sh py launch_split tools/launch_split.py       # launch_split.json
bash tools/gpu/run.sh sweep small2 --only small --reps 11         # small.json
bash tools/gpu/run.sh sweep xcd_v --only vknob --key 49 --values 0,1 --reps 9                       # tile_xcd_varlen.json
bash tools/gpu/run.sh sweep xcd_ops --only opsknob --key 49 --values 0,1 --encode-L 1472,1024,256,64 --reps 11   # tile_xcd_ops.json
bash tools/gpu/run.sh sweep enc_xcd --only opsknob --key 5 --values 1,0 --encode-L 1472,1024,512,256,64 --reps 11  # encode_xcd.json
bash tools/gpu/run.sh sweep ragged --only ragged --reps 9          # ragged.json
bash tools/gpu/run.sh py e2e tools/e2e_sweep.py                    # e2e.json
# N = 2 rehearsal on one GPU (gloo), bench_n2_share_device.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --share-device --steps 10 --warmup 2
# session 3 of round 2: where the headline's last 8% goes (profiles/r02/headline/)
bash tools/gpu/run.sh py launch_length tools/launch_length.py                       # launch_length.json
bash tools/gpu/run.sh py xcd_orders tools/launch_length.py --orders --rounds 3 --reps 10   # xcd_orders.json
bash tools/gpu/run.sh py tile_timeline tools/tile_timeline.py                       # tile_timeline.json
bash tools/gpu/run.sh py tile_timeline2 tools/tile_timeline.py --no-16m --save gpurun_out/tt --percu 4,6,0   # tile_timeline_percu.json
bash tools/gpu/run.sh py tile_phases tools/tile_timeline.py --no-16m --percu 0      # tile_phases.json
bash tools/gpu/run.sh py tile_phases_early tools/tile_timeline.py --no-16m --early   # tile_phases_early_table.json
bash tools/gpu/run.sh py sustained tools/sustained.py --n 300                       # sustained.json
bash tools/gpu/run.sh py sustained2 tools/sustained.py --n 100 --variants           # sustained_variants.json
bash tools/gpu/run.sh py power tools/power_probe.py                                 # power_encode_vs_copy.json
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT -f csv -d gpurun_out/clk -o run -- python3 tools/sustained.py --n 100   # sclk_encode_vs_copy.json
bash tools/gpu/run.sh sweep early --only knob --key 30 --values=-1,1,0 --encode-L 1472 --reps 15    # early_table_1472.json
bash tools/gpu/run.sh sweep regsum --only knob --key 56 --values=0,1 --encode-L 1472,1024 --reps 15  # regsum_1472_1024.json (form removed)
bash tools/gpu/run.sh sweep small1 --only small --reps 7                            # small_onepass/ (form removed)
bash tools/gpu/run.sh py small_timeline tools/small_timeline.py                     # small_onepass/timeline_xcd_order.json
# end-of-round refresh
bash tools/gpu/run.sh tests && bash tools/gpu/run.sh smoke && bash tools/gpu/run.sh bench r02j
bash tools/gpu/run.sh trace enc1M bench.py --no-legs --no-cpu-baseline
bash tools/gpu/run.sh pmc enc1M bench.py --no-legs --no-cpu-baseline --steps 10 --warmup 2
bash tools/gpu/run.sh sweep tabdma --only knob --key 30 --values=-1,2,1 --encode-L 1472,1024,512 --reps 15   # table_dma.json
bash tools/gpu/run.sh sweep tabdma2 --only knob --key 30 --values=-1,2 --encode-L 1472,512,768 --reps 25   # table_dma_repeat.json
bash tools/gpu/run.sh tests && bash tools/gpu/run.sh smoke && bash tools/gpu/run.sh bench r02k   # after the table-by-DMA default
bash tools/gpu/run.sh py tile_phases_dma tools/tile_timeline.py --no-16m   # tile_phases_table_dma.json
bash tools/gpu/run.sh trace enc16M tools/run_kernel.py --op encode --n 16777216 --steps 20 && bash tools/gpu/run.sh pmc enc16M tools/run_kernel.py --op encode --n 16777216 --steps 5   # encode_16Mx1472_summary.json (refresh)
bash tools/gpu/run.sh tests && bash tools/gpu/run.sh smoke && bash tools/gpu/run.sh bench r02l   # final tree (XCD sweep forms removed): 204 GPU tests
