"""Per-dispatch / per-wave SQ counters of the step or rollout kernel from scripts/gpu_sq.sh passes.
    python sq_summarize.py OUTDIR TAG TASK N MODE   -> OUTDIR/sq_TAG_TASK_N_MODE_summary.json"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    out, tag, task, n, mode = sys.argv[1:6]
    kname = "quad_rollout_kernel<" if mode == "rollout" else "quad_step_kernel<"
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(out, f"sq_{tag}_{task}_{n}_{mode}_p*", "**", "*counter_collection.csv"),
                       recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name", "")
                if kname in name or (mode != "rollout" and "quad_step_pipe_kernel<" in name):
                    vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
    res = {"task": task, "num_envs": int(n), "mode": mode, "kernel": kname.rstrip("<"),
           "steps_per_launch": 16 if mode == "rollout" else 1}
    for c, v in sorted(vals.items()):
        res[c] = sum(v) / len(v)
        res[c + "_dispatches"] = len(v)
    w = res.get("SQ_WAVES")
    if w:
        for c in list(vals):
            if c != "SQ_WAVES":
                res[c + "_per_wave"] = res[c] / w
                res[c + "_per_wave_step"] = res[c] / w / res["steps_per_launch"]
    path = os.path.join(out, f"sq_{tag}_{task}_{n}_{mode}_summary.json")
    with open(path, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in res.items()
                      if "per_wave_step" in k or k in ("task", "num_envs", "mode")}))


if __name__ == "__main__":
    main()
