#!/bin/bash
# bench.py's timed region (scripts/exp/region_breakdown.py) by the timing events' creation flags, and without
# them.  Output: gpurun_out/region_events.jsonl
set -u
O=gpurun_out/region_events.jsonl
: > $O
for F in "" 0 0x20000000 0x40000000 0x60000000; do
  timeout -k 10 120 python -u scripts/exp/region_breakdown.py LeeLanded 4096 sync,noev,empty,sync,noev,empty $F >> $O || exit 1
done
cat $O
