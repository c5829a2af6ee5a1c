"""Average per-dispatch value of PMC counters of the single-step kernel (quad_step_kernel<T>; the fused rollout is quad_rollout_kernel<T>).
python counters_summarize.py OUTDIR TAG TASK N COUNTER...  -> OUTDIR/cnt_TAG_TASK_N_summary.json"""
import csv
import glob
import json
import os
import sys


def main():
    out, tag, task, n = sys.argv[1:5]
    res = {"task": task, "num_envs": int(n)}
    for c in sys.argv[5:]:
        vals = []
        for f in glob.glob(os.path.join(out, f"cnt_{tag}_{task}_{n}_{c}", "**", "*counter_collection.csv"),
                           recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    name = row.get("Kernel_Name", "")
                    if "quad_step_kernel<" in name and row.get("Counter_Name") == c:
                        vals.append(float(row["Counter_Value"]))
        res[c] = sum(vals) / len(vals) if vals else None
    if res.get("SQ_WAVES"):
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES"):
            if res.get(c) is not None:
                res[c + "_per_wave"] = res[c] / res["SQ_WAVES"]
    with open(os.path.join(out, f"cnt_{tag}_{task}_{n}_summary.json"), "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
