#!/bin/bash
# Round-4 batch: GPU suite on the in-tree library, A/B against a previous build (latency-regime configs and the
# large-N estimator rollouts), the statistics-tail probe, the driver's bench command.
#   bash scripts/archive/r04_batch2.sh PREV.so TAG
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
P=$1; TAG=$2
O="$R/gpurun_out"
mkdir -p "$O"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > "$O/pytest_gpu_$TAG.log" 2>&1
rc=$?; tail -3 "$O/pytest_gpu_$TAG.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u scripts/exp/lib_ab.py "$P" ouzelum_amd/libouzelum_hip.so 3 > "$O/lib_ab_$TAG.jsonl" 2> "$O/lib_ab_$TAG.err" || { echo "lib_ab failed"; tail -5 "$O/lib_ab_$TAG.err"; exit 1; }
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
timeout -k 10 900 bash scripts/archive/large_n_lib_ab.sh "$P" "QuadTracking QuadMixed EKFLeeLanded" "4194304" 2>&1 | grep -v amdgpu.ids > "$O/large_n_ab_$TAG.txt" || exit 1
grep rollout "$O/large_n_ab_$TAG.txt"
timeout -k 10 300 python scripts/exp/stats_tail_probe.py 2>&1 | grep -v amdgpu.ids > "$O/stats_tail_$TAG.jsonl" || exit 1
cat "$O/stats_tail_$TAG.jsonl"
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --detail "$O/bench_detail_driver_args_$TAG.json" \
  > "$O/bench_driver_args_$TAG.json" 2> "$O/bench_driver_args_$TAG.err" || { echo "bench failed"; tail -5 "$O/bench_driver_args_$TAG.err"; exit 1; }
head -c 600 "$O/bench_driver_args_$TAG.json"
