#!/bin/bash
# Round 5: the mixed curriculum as one launch per task above the latency regime -- its parity tests, then the
# per-step A/B (one launch per task against one launch).
set -u
O=gpurun_out/r05m
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_timed_kernels.py -m gpu -q -x -k "mixed_split or large_n_fused" \
  --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.out 2>&1 || { tail -40 $O/pytest.out; exit 1; }
tail -2 $O/pytest.out
timeout -k 10 400 python -u scripts/exp/mixed_step_split_ab.py 3 > $O/step_ab.jsonl 2> $O/step_ab.err || { tail -5 $O/step_ab.err; exit 1; }
cat $O/step_ab.jsonl
