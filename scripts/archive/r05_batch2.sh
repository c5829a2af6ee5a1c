#!/bin/bash
# Round-5 batch 2: A/B of the f64 EKF (product) against the round-4 f32 EKF (-DOUZ_EKF_F32), and of the statistics
# hand-off with an agent-scope acquire (-DOUZ_STATS_ACQUIRE); then the GPU suite.   bash scripts/archive/r05_batch2.sh
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O="$R/gpurun_out/r05b2"
mkdir -p "$O"
cd "$R"
for V in ekff32 acq; do
  timeout -k 10 600 python -u scripts/exp/lib_ab.py ouzelum_amd/libouzelum_hip.so ouzelum_amd/libouzelum_$V.so 3 \
    > "$O/lib_ab_$V.jsonl" 2> "$O/lib_ab_$V.err" || { echo "lib_ab $V failed"; tail -5 "$O/lib_ab_$V.err"; exit 1; }
  python3 - "$O/lib_ab_$V.jsonl" <<'PY'
import json, sys, collections
rows = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")]
agg = collections.defaultdict(list)
for r in rows:
    if "config" in r:
        agg[(r["lib"].split("/")[-1], r["config"])].append((r["fused_us_per_step"], r.get("per_step_us"), r["state_sha16"], r.get("step_state_sha16")))
for k in sorted(agg):
    v = agg[k]
    print(k, "fused", sorted(x[0] for x in v), "step", sorted(x[1] for x in v), "sha", {x[2] for x in v}, {x[3] for x in v})
PY
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 450 --timeout-method thread -p no:cacheprovider \
  > "$O/gpu_suite.log" 2>&1; rc=$?
tail -5 "$O/gpu_suite.log"
exit $rc
