#!/bin/bash
# scripts/archive/sync_latency.hip under the device schedule flags and the runtime's active-wait knob.
set -u
O=gpurun_out/sync_latency.jsonl
hipcc --offload-arch=gfx950 -O3 -o /tmp/sync_latency scripts/archive/sync_latency.hip 2>/dev/null || exit 1
: > $O
for m in default spin yield block; do timeout -k 10 60 /tmp/sync_latency $m >> $O || exit 1; done
ROC_ACTIVE_WAIT_TIMEOUT=200 timeout -k 10 60 /tmp/sync_latency default | sed 's/"default"/"default+ROC_ACTIVE_WAIT_TIMEOUT=200"/' >> $O || exit 1
ROC_ACTIVE_WAIT_TIMEOUT=5000 timeout -k 10 60 /tmp/sync_latency default | sed 's/"default"/"default+ROC_ACTIVE_WAIT_TIMEOUT=5000"/' >> $O || exit 1
cat $O
