#!/bin/bash
# Address-translation counters of the per-step kernel at two sizes (explains the 4 M -> 16 M HBM-fraction
# drop of LeeLanded at identical PMC bytes): lists the UTCL/TLB counters the box offers, then one TCP pass
# per size with the UTCL1 request / miss counters (kernel trace only, <= 4 TCP counters per pass).
#   bash scripts/gpu_tlb.sh TAG TASK "SIZES" [LAUNCHES]
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; TASK=$2; SIZES=$3; L=${4:-20}
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 60 rocprofv3 -L > "$R/gpurun_out/counters_${TAG}.txt" 2>&1 || true
grep -iE "UTCL|TLB|UTC" "$R/gpurun_out/counters_${TAG}.txt" | head -40
P=${PMC:-"TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_PERMISSION_MISS_sum"}
for N in $SIZES; do
  D="$R/gpurun_out/tlb_${TAG}_${TASK}_${N}"
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P -d "$D" -o run --output-format csv -- \
    python3 "$R/scripts/kernel_driver.py" --task "$TASK" --num-envs "$N" --mode step --launches "$L" \
    > "$D.log" 2>&1 || { echo "pass $N failed"; tail -5 "$D.log"; exit 1; }
  python3 - "$D" "$N" <<'PY'
import csv, glob, sys
from collections import defaultdict
d, n = sys.argv[1], int(sys.argv[2])
v = defaultdict(list)
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if "quad_step" in row.get("Kernel_Name", ""):
            v[row["Counter_Name"]].append(float(row["Counter_Value"]))
print(n, {k: round(sum(x) / len(x)) for k, x in v.items()}, {k + "_per_env": round(sum(x) / len(x) / n, 3) for k, x in v.items()})
PY
done
