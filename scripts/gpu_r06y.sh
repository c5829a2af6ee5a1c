#!/bin/bash
# Round 6, final tree: the driver's bench command three times (run-to-run spread of the headline), then the N = 8
# command form rehearsed with 8 gloo ranks sharing the one GPU (the RCCL form needs 8 devices: the driver's node).
set -o pipefail
O=gpurun_out/r06y
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 --detail $O/detail_$i.json > $O/bench_$i.out 2> $O/bench_$i.err || exit 1
  tail -n 1 $O/bench_$i.out | cut -c1-200
done
OUZ_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 8 --steps 20 --warmup 5 > $O/bench_gloo_8.out 2> $O/bench_gloo_8.err || exit 1
tail -c 400 $O/bench_gloo_8.out
