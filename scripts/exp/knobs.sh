#!/bin/bash
# HIP runtime launch knobs vs per-step host/GPU cost (probe only, not part of the product).
set -u
for kv in "" "HIP_FORCE_DEV_KERNARG=0" "HIP_FORCE_DEV_KERNARG=1" "AMD_DIRECT_DISPATCH=0" \
          "DEBUG_CLR_KERNARG_HDP_FLUSH_WA=0" "DEBUG_CLR_KERNARG_HDP_FLUSH_WA=1" "ROC_USE_FGS_KERNARG=1" \
          "ROC_SYSTEM_SCOPE_SIGNAL=0" "ROC_CPU_WAIT_FOR_SIGNAL=0"; do
  echo "== ${kv:-default}"
  env $kv timeout -k 10 60 ./examples/c_host_step || exit 1
  env $kv timeout -k 10 60 ./scripts/exp/launch_cost || exit 1
done
