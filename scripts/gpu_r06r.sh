#!/bin/bash
# Round 6: the N > 1 bench path rehearsed on one GPU (two and four ranks sharing the device over gloo, the driver's
# torchrun command form), on the final tree.  The RCCL form needs one device per rank: the driver's 8-GPU node.
set -o pipefail
O=gpurun_out/r06r
mkdir -p $O
for n in 2 4; do
  OUZ_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port 2951$n bench.py --gpus $n --steps 20 --warmup 5 > $O/bench_gloo_$n.out 2> $O/bench_gloo_$n.err || exit 1
  tail -c 600 $O/bench_gloo_$n.out; echo
done
