#!/bin/bash
# Round 5: the estimator tasks' per-step kernel above the latency regime at 3 / 4 waves per SIMD (OUZ_EST_STEP_WPE
# variant builds) against the product build; large_n_lib_ab.py, interleaved rounds.
set -u
O=gpurun_out/r05w
mkdir -p $O
L=ouzelum_amd
for v in 3 4; do
  timeout -k 10 500 python -u scripts/archive/large_n_lib_ab.py $L/libouzelum_hip.so $L/libouzelum_swpe$v.so 2 \
    QuadTracking:4194304 EKFLeeLanded:4194304 QuadMixed:4194304 QuadTracking:16777216 > $O/ab_wpe$v.jsonl 2> $O/ab_wpe$v.err \
    || { tail -5 $O/ab_wpe$v.err; exit 1; }
  cat $O/ab_wpe$v.jsonl
done
