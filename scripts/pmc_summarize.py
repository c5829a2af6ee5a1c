"""Average FETCH_SIZE / WRITE_SIZE (KB) per quad_step_kernel (or quad_rollout_kernel) dispatch -> HBM bytes
per launch, plus the kernel's average duration from a --kernel-trace --stats pass of the same workload.

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports 1/2 of the bytes of wide
coalesced streaming reads -> doubled; WRITE_SIZE is exact for 16-B streaming stores.
Writes profiles-ready JSON next to the raw counters:
    python pmc_summarize.py OUTDIR TAG TASK N            (round-1 layout: pmc_TAG_TASK_N_*, step kernel)
    python pmc_summarize.py OUTDIR TAG TASK N MODE [K]   (scripts/gpu_pmc2.sh / gpu_roofline_evidence.sh:
                                                          pmc_TAG_MODE_TASK_N_*; K: the rollout's launch length)
A rollout of a task that streams it at this size (bench.py streamed_rollout) runs step kernels: its summary
is the step kernel's.  ``lib_sha16``: the library the counters were taken on (bench.py only uses a summary of
the library it loaded).
"""
import csv
import glob
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def lib_sha16(path=None):
    """The library's source id (ouz_source_id(): its sources and build flags, stable across rebuilds), or for a
    library without one, the sha256 of its bytes.  PMC / VALU summaries carry it; bench.py prices evidence only
    from summaries of the library it loaded."""
    import ctypes
    path = path or os.environ.get("OUZ_LIB") or os.path.join(ROOT, "ouzelum_amd", "libouzelum_hip.so")
    try:
        lib = ctypes.CDLL(path)
        fn = lib.ouz_source_id
        fn.restype = ctypes.c_char_p
        sid = fn().decode()
        if sid and sid != "unknown":
            return "src-" + sid
    except (OSError, AttributeError):
        pass
    with open(path, "rb") as fh:
        return hashlib.sha256(fh.read()).hexdigest()[:16]


def _hit(name, kernel):
    # the single-step launch (quad_step_kernel<TASK>, or its large-N pipelined form quad_step_pipe_kernel<TASK>),
    # not quad_rollout_kernel<TASK>
    return kernel in name or (kernel == "quad_step_kernel<" and "quad_step_pipe_kernel<" in name)


def avg_counter(path_glob, counter, kernel="quad_step_kernel<"):
    vals = []
    for f in glob.glob(path_glob, recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if _hit(row.get("Kernel_Name", ""), kernel) and row.get("Counter_Name") == counter:
                    vals.append(float(row["Counter_Value"]))
    return (sum(vals) / len(vals), len(vals)) if vals else (None, 0)


def avg_duration_us(stats_dir, kernel):
    """Average duration of the kernel from the rocprofv3 --stats kernel_stats.csv (ns -> us)."""
    for f in glob.glob(os.path.join(stats_dir, "**", "*kernel_stats.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if _hit(row.get("Name", ""), kernel):
                    return float(row["AverageNs"]) / 1e3, int(row["Calls"]), os.path.relpath(f, stats_dir)
    return None, 0, None


def _env_work(name, marker):
    # the dispatches of the workload: per step, the three tasks' step kernels; per rollout, also the streamed tasks'
    # step launches, the last-row copies and the statistics launch -- not the env's creation (init_state_kernel)
    # nor torch's set-up kernels (the action ring's rand, zero fills)
    if marker.startswith("quad_step_kernel<"):
        return "quad_step_kernel<" in name
    return any(k in name for k in ("quad_rollout_kernel<", "quad_step_kernel<", "episode_stats",
                                   "__amd_rocclr_copyBuffer"))


def mixed_split_counter(path_glob, counter, marker):
    """The mixed curriculum above the latency regime runs one launch per task (quad_kernels.hip mix_split; a rollout
    also runs its streamed tasks' step launches, the last-row copies and an episode-statistics launch): the summed
    counter of all the env's dispatches per launch of the marker kernel (the QuadTracking chunks' kernel, one per
    step or per rollout launch)."""
    tot, marks = 0.0, 0
    for f in glob.glob(path_glob, recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name", "")
                if row.get("Counter_Name") != counter or not _env_work(name, marker):
                    continue
                tot += float(row["Counter_Value"])
                marks += marker in name
    return (tot / marks, marks) if marks else (None, 0)


def mixed_split_duration_us(stats_dir, marker):
    """Summed rocprof duration of the env's dispatches per launch of the marker kernel."""
    for f in glob.glob(os.path.join(stats_dir, "**", "*kernel_stats.csv"), recursive=True):
        with open(f) as fh:
            rows = list(csv.DictReader(fh))
        marks = sum(int(r["Calls"]) for r in rows if marker in r.get("Name", ""))
        if marks:
            tot = sum(float(r["TotalDurationNs"]) for r in rows if _env_work(r.get("Name", ""), marker))
            return tot / marks / 1e3, marks, os.path.relpath(f, stats_dir)
    return None, 0, None


def main():
    out, tag, task, n = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
    mode = sys.argv[5] if len(sys.argv) > 5 else None
    base = os.path.join(out, f"pmc_{tag}_{mode}_{task}_{n}" if mode else f"pmc_{tag}_{task}_{n}")
    streamed = mode == "rollout" and n > 131072 and task not in ("EKFLeeLanded", "QuadTracking", "QuadMixed")
    kernel = "quad_rollout_kernel<" if mode == "rollout" and not streamed else "quad_step_kernel<"
    # VecTask.step of the mixed curriculum above the latency regime is one launch per task (the default); its fused
    # rollout one launch unless OUZ_MIXED_SPLIT_ROLLOUT=1
    split = (task == "QuadMixed" and n > 65536 and os.environ.get("OUZ_MIXED_SPLIT", "1") != "0"
             and (mode != "rollout" or os.environ.get("OUZ_MIXED_SPLIT_ROLLOUT", "0") != "0"))
    marker = kernel + "3,"   # the QuadTracking chunks' kernel (OUZ_TASK_TRACKING = 3)
    if split:
        fetch, nf = mixed_split_counter(base + "_FETCH_SIZE/**/*counter_collection.csv", "FETCH_SIZE", marker)
        write, nw = mixed_split_counter(base + "_WRITE_SIZE/**/*counter_collection.csv", "WRITE_SIZE", marker)
    else:
        fetch, nf = avg_counter(base + "_FETCH_SIZE/**/*counter_collection.csv", "FETCH_SIZE", kernel)
        write, nw = avg_counter(base + "_WRITE_SIZE/**/*counter_collection.csv", "WRITE_SIZE", kernel)
    steps = 1
    if kernel == "quad_rollout_kernel<":   # kernel_driver.py's --launch-steps (default bench.evidence_launch_steps)
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from bench import evidence_launch_steps
        steps = int(sys.argv[6]) if len(sys.argv) > 6 else evidence_launch_steps(n)
    res = {"task": task, "num_envs": n, "kernel": kernel.rstrip("<"), "steps_per_launch": steps,
           "dispatches": [nf, nw], "fetch_size_kb_raw": fetch, "write_size_kb": write}
    try:
        res["lib_sha16"] = lib_sha16()
    except OSError:
        pass
    if split:
        res["mixed_split"] = ("per launch: every env dispatch (the three tasks' kernels, the streamed tasks' step "
                              "launches, copies, statistics) summed over the QuadTracking chunks' launches")
    us, calls, src = (mixed_split_duration_us if split else avg_duration_us)(base + "_STATS", marker if split else kernel)
    if us is not None:
        res.update({"rocprof_avg_us": us, "rocprof_calls": calls, "rocprof_stats_csv": src})
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
