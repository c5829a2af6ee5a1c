#!/bin/bash
# A/B of a library variant on the large-N sweep entries (bench.sweep_entries: step kernel + fused / streamed
# rollout, HIP events around back-to-back launches): product build and OUZ_LIB=$1 alternating twice.
#   bash scripts/archive/large_n_lib_ab.sh VARIANT.so "QuadTracking QuadMixed" "4194304"
set -u
cd "$(dirname "$0")/../.."
V=$1; TASKS=$2; SIZES=$3
for r in 1 2; do
  for L in ouzelum_amd/libouzelum_hip.so "$V"; do
    for T in $TASKS; do
      for N in $SIZES; do
        echo "# $L round $r"
        OUZ_ALLOW_INSTRUMENTED=1 OUZ_LIB=$PWD/$L timeout -k 10 300 python -u scripts/exp/rollout_largeN.py "$T" "$N" || exit 1
      done
    done
  done
done
