#!/bin/bash
# Round 6: launch-count trims of the learner's data movement, measured (scripts/exp/copy_gather_probe.py, 3 rounds).
set -o pipefail
mkdir -p gpurun_out/r06u
for i in 1 2 3; do timeout -k 10 120 python scripts/exp/copy_gather_probe.py >> gpurun_out/r06u/probe.jsonl || exit 1; done
cat gpurun_out/r06u/probe.jsonl
