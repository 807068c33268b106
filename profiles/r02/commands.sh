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
