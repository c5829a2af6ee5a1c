#!/bin/bash
# Build and run scripts/exp/emit_pattern.hip on the GPU box: plain timing, a WRITE_SIZE pass and a
# --kernel-trace --stats pass; summary JSON lines in gpurun_out/emit_pattern/summary.jsonl.
#   bash scripts/archive/emit_pattern.sh [envs] [sleep]
set -eu
R=${GRAFT_REPO_ROOT:-$(pwd)}
N=${1:-4096}; S=${2:-1}
O="$R/gpurun_out/emit_pattern"
mkdir -p "$O"
export TMPDIR=/tmp
hipcc --offload-arch=gfx950 -O3 -o /tmp/emit_pattern "$R/scripts/exp/emit_pattern.hip" 2> "$O/build.log"
cd /tmp
timeout -k 10 60 /tmp/emit_pattern "$N" "$S" > "$O/timing.jsonl"
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$O/write" -o run --output-format csv -- \
  /tmp/emit_pattern "$N" "$S" > "$O/write.log" 2>&1
timeout -k 10 60 rocprofv3 --kernel-trace --stats -d "$O/stats" -o run --output-format csv -- \
  /tmp/emit_pattern "$N" "$S" > "$O/stats.log" 2>&1
python3 - "$O" "$N" <<'PY'
import csv, glob, json, sys
o, n = sys.argv[1], int(sys.argv[2])
w = {}
for f in glob.glob(o + "/write/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if row.get("Counter_Name") == "WRITE_SIZE":
            w.setdefault("class" if "emit_pattern<1>" in row["Kernel_Name"] else "identity", []).append(float(row["Counter_Value"]))
st = {}
for f in glob.glob(o + "/stats/**/*kernel_stats.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        st["class" if "emit_pattern<1>" in row["Name"] else "identity"] = float(row["AverageNs"]) / 1e3
with open(o + "/summary.jsonl", "w") as fh:
    for k, v in sorted(w.items()):
        kb = sum(v) / len(v)
        r = {"layout": k, "envs": n, "dispatches": len(v), "write_size_kb": round(kb, 1),
             "write_bytes_per_env_step": round(kb * 1024 / (n * 16), 2), "algorithmic": 65,
             "rocprof_avg_us": st.get(k)}
        fh.write(json.dumps(r) + "\n")
        print(json.dumps(r))
PY
cat "$O/timing.jsonl"
