#!/bin/bash
# Build and run scripts/exp/step_emit_pattern.hip on the GPU box: timing (both layouts interleaved), WRITE_SIZE and
# FETCH_SIZE passes (separate runs); summary JSON lines in gpurun_out/step_emit_pattern/summary.jsonl.
#   bash scripts/archive/step_emit_pattern.sh [envs] [sleep]
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
N=${1:-4096}; S=${2:-2}
O="$R/gpurun_out/step_emit_pattern"
mkdir -p "$O"
export TMPDIR=/tmp
hipcc --offload-arch=gfx950 -O3 -o /tmp/step_emit_pattern "$R/scripts/exp/step_emit_pattern.hip" 2> "$O/build.log"
cd /tmp
timeout -k 10 60 /tmp/step_emit_pattern "$N" "$S" 5 > "$O/timing.jsonl"
for C in WRITE_SIZE FETCH_SIZE; do
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $C -d "$O/$C" -o run --output-format csv -- \
    /tmp/step_emit_pattern "$N" "$S" 1 > "$O/$C.log" 2>&1
done
python3 - "$O" "$N" <<'PY'
import csv, glob, json, sys
o, n = sys.argv[1], int(sys.argv[2])
out = {}
for c in ("WRITE_SIZE", "FETCH_SIZE"):
    for f in glob.glob(f"{o}/{c}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") == c:
                k = "class" if "step_emit<1>" in row["Kernel_Name"] else "identity"
                out.setdefault(k, {}).setdefault(c, []).append(float(row["Counter_Value"]))
with open(o + "/summary.jsonl", "w") as fh:
    for k, d in sorted(out.items()):
        w = sum(d["WRITE_SIZE"]) / len(d["WRITE_SIZE"]); f = sum(d["FETCH_SIZE"]) / len(d["FETCH_SIZE"])
        r = {"layout": k, "envs": n, "write_bytes_per_env": round(w * 1024 / n, 2),
             "fetch_bytes_per_env_raw": round(f * 1024 / n, 2), "algorithmic": {"read": 9, "write": 65}}
        fh.write(json.dumps(r) + "\n"); print(json.dumps(r))
PY
cat "$O/timing.jsonl"
