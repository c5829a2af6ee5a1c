#!/bin/bash
# bench.py's timed region (scripts/exp/region_breakdown.py, torch.cuda.synchronize variant) under the HIP runtime's
# launch / wait knobs, one process each.  Output: gpurun_out/region_knobs.jsonl
set -u
O=gpurun_out/region_knobs.jsonl
: > $O
run() { env "$@" timeout -k 10 120 python -u scripts/exp/region_breakdown.py LeeLanded 4096 sync,empty,sync,empty >> $O || exit 1; }
run X=0
run HIP_FORCE_DEV_KERNARG=1
run HIP_FORCE_DEV_KERNARG=0
run ROC_ACTIVE_WAIT_TIMEOUT=1000
run ROC_ACTIVE_WAIT_TIMEOUT=0
run ROC_SYSTEM_SCOPE_SIGNAL=0
run ROC_CPU_WAIT_FOR_SIGNAL=0
run ROC_USE_FGS_KERNARG=1
cat $O
