# round 3: N = 8 rehearsal on one GPU (8 ranks sharing cuda:0 over gloo), the driver's torchrun form
set -e
O=gpurun_out
timeout -k 20 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 8 --share-device --steps 10 --warmup 2 > $O/bench_n8_share.json 2> $O/bench_n8_share.err
echo done
