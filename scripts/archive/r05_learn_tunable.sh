#!/bin/bash
# Round 5 probe: PyTorch TunableOp (per-shape selection among hipBLASLt / rocBLAS GEMM solutions) on the learner's
# GEMMs, config D.  Tuning run (results written), then interleaved runs reading the tuned file vs TunableOp off.
set -u
O=gpurun_out/r05t
mkdir -p $O
B="scripts/bench_learner.py --env QuadFault --num_envs 8192 --iters 40"
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=$O/tunableop_results%d.csv \
  timeout -k 10 500 python -u $B --warmup 8 > $O/tune.json 2> $O/tune.err || { tail -20 $O/tune.err; exit 1; }
echo "tuning run: $(cat $O/tune.json)"
ls -la $O
for r in 1 2 3; do
  timeout -k 10 300 python -u $B --warmup 5 > $O/off_$r.json 2> $O/off_$r.err || { tail -5 $O/off_$r.err; exit 1; }
  echo "off round $r: $(cat $O/off_$r.json)"
  PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=$O/tunableop_results%d.csv \
    timeout -k 10 300 python -u $B --warmup 5 > $O/on_$r.json 2> $O/on_$r.err || { tail -5 $O/on_$r.err; exit 1; }
  echo "tuned round $r: $(cat $O/on_$r.json)"
done
