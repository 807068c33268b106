# round 3 final tree: N = 2 rehearsal (2 ranks sharing cuda:0 over gloo), the driver's torchrun form
set -e
O=gpurun_out
timeout -k 20 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29519 bench.py --gpus 2 --share-device --steps 10 --warmup 2 > $O/bench_n2_share_final.json 2> $O/bench_n2_share_final.err
echo done
