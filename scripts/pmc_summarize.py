"""Average FETCH_SIZE / WRITE_SIZE (KB) per quad_step_kernel (or quad_rollout_kernel) dispatch -> HBM bytes
per launch.

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports 1/2 of the bytes of wide
coalesced streaming reads -> doubled; WRITE_SIZE is exact for 16-B streaming stores.
Writes profiles-ready JSON next to the raw counters:
    python pmc_summarize.py OUTDIR TAG TASK N            (round-1 layout: pmc_TAG_TASK_N_*, step kernel)
    python pmc_summarize.py OUTDIR TAG TASK N MODE       (scripts/gpu_pmc2.sh: pmc_TAG_MODE_TASK_N_*)
"""
import csv
import glob
import json
import os
import sys


def avg_counter(path_glob, counter, kernel="quad_step_kernel<"):
    vals = []
    for f in glob.glob(path_glob, recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name", "")
                # the single-step launch (quad_step_kernel<TASK>, or its large-N pipelined form
                # quad_step_pipe_kernel<TASK>), not quad_rollout_kernel<TASK>
                hit = kernel in name or (kernel == "quad_step_kernel<" and "quad_step_pipe_kernel<" in name)
                if hit and row.get("Counter_Name") == counter:
                    vals.append(float(row["Counter_Value"]))
    return (sum(vals) / len(vals), len(vals)) if vals else (None, 0)


def main():
    out, tag, task, n = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
    mode = sys.argv[5] if len(sys.argv) > 5 else None
    base = os.path.join(out, f"pmc_{tag}_{mode}_{task}_{n}" if mode else f"pmc_{tag}_{task}_{n}")
    kernel = "quad_rollout_kernel<" if mode == "rollout" else "quad_step_kernel<"
    fetch, nf = avg_counter(base + "_FETCH_SIZE/**/*counter_collection.csv", "FETCH_SIZE", kernel)
    write, nw = avg_counter(base + "_WRITE_SIZE/**/*counter_collection.csv", "WRITE_SIZE", kernel)
    steps = 16 if mode == "rollout" else 1
    res = {"task": task, "num_envs": n, "kernel": kernel.rstrip("<"), "steps_per_launch": steps,
           "dispatches": [nf, nw], "fetch_size_kb_raw": fetch, "write_size_kb": write}
    if fetch is not None and write is not None:
        res["read_bytes_corrected"] = fetch * 1024 * 2
        res["write_bytes"] = write * 1024
        res["traffic_bytes_per_launch"] = res["read_bytes_corrected"] + res["write_bytes"]
        res["traffic_bytes_per_env_step"] = res["traffic_bytes_per_launch"] / (n * steps)
    with open(base + "_summary.json", "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
