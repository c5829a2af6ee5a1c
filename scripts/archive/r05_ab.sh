#!/bin/bash
# Round-5 A/B of the product library against a variant build (scripts/exp/lib_ab.py, 3 interleaved rounds).
#   bash scripts/archive/r05_ab.sh VARIANT.so TAG
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
V=$1; TAG=$2
O="$R/gpurun_out/r05ab"
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u scripts/exp/lib_ab.py ouzelum_amd/libouzelum_hip.so "$V" 3 \
  > "$O/lib_ab_$TAG.jsonl" 2> "$O/lib_ab_$TAG.err" || { echo "lib_ab $TAG failed"; tail -5 "$O/lib_ab_$TAG.err"; exit 1; }
python3 - "$O/lib_ab_$TAG.jsonl" <<'PY'
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
