#!/usr/bin/env python3
"""Markdown tables for DESIGN.md §5.3 from a bench.py side file (``--detail``): every roofline entry the run
priced (headline, per-step path, the other configs, the large-N sweeps), with its algorithmic bytes, the PMC
traffic of the committed summary of the same library build, the live and rocprof-priced fractions, and the
issue-bound view where a VALU summary of that build exists.

    python scripts/evidence_tables.py gpurun_out/r04d/bench_detail_default.json
"""
import json
import sys


def entries(d):
    """(label, roofline entry) for every priced workload in the side file."""
    task = d["config"]["task"]
    yield f"{task} (headline)", d["roofline"]
    if d.get("per_step_launch"):
        yield f"{task} (headline)", d["per_step_launch"]["roofline"]
    for e in d.get("roofline_sweep") or []:
        yield task, e
    for c in d.get("configs") or []:
        yield f"{c['task']} ({c['config']})", c["roofline"]
        if c.get("per_step_launch"):
            yield f"{c['task']} ({c['config']})", c["per_step_launch"]["roofline"]
        for e in c.get("roofline_sweep") or []:
            yield c["task"], e


def fmt(x, nd=3):
    if x is None:
        return "-"
    if isinstance(x, float):
        return f"{x:.{nd}f}"
    return str(x)


def roofline_table(d):
    rows = ["| workload | kernel | envs | steps/launch | µs/step | alg. B/env-step | PMC B/env-step (read + write) "
            "| PMC / alg. | frac (HIP events) | frac (rocprof avg) |",
            "|---|---|---|---|---|---|---|---|---|---|"]
    for label, e in entries(d):
        td = e.get("traffic_detail") or {}
        pmc = td.get("bytes_per_env_step")
        rw = (f"{pmc:.1f} ({td['read_bytes_per_env_step']:.1f} + {td['write_bytes_per_env_step']:.1f})"
              if pmc is not None else ("stale" if td.get("stale") else "-"))
        # PMC traffic against the algorithmic bytes of the SAME launch (the summary's own launch length: bench.py
        # price_summary), not of the priced region's launches
        ratio = e.get("traffic_alg_ratio") or (pmc / e["bytes_per_env_step"] if pmc else None)
        kern = e["kernel"].replace("quad_", "").replace("_kernel", "")
        if e.get("steps_per_rollout"):
            kern = "rollout (streamed step launches)"
        rows.append(f"| {label} | {kern} | {e['num_envs']} | {e.get('steps_per_launch', 1)} | "
                    f"{fmt(e['kernel_us'])} | {fmt(e['bytes_per_env_step'], 1)} | {rw} | {fmt(ratio, 2)} | "
                    f"{fmt(e['frac'], 4)} | {fmt(e.get('frac_from_rocprof_avg'), 4)} |")
    return "\n".join(rows)


def issue_table(d):
    rows = ["| workload | kernel | envs | µs/step | VALU issue frac | VALU active frac | issue active frac | "
            "wait frac | SIMD frac | chip VALU frac | f64 share | µs from counters / launch | rocprof avg µs / launch | "
            "counters / rocprof |",
            "|---|---|---|---|---|---|---|---|---|---|---|---|---|---|"]
    for label, e in entries(d):
        iss = e.get("issue")
        if not iss:
            continue
        kern = e["kernel"].replace("quad_", "").replace("_kernel", "")
        rp = (e.get("traffic_detail") or {}).get("rocprof_kernel_us_per_launch")
        ratio = iss["kernel_us_from_counters"] / rp if rp else None
        rows.append(f"| {label} | {kern} | {e['num_envs']} | {fmt(e['kernel_us'])} | {fmt(iss['valu_issue_frac'])} | "
                    f"{fmt(iss['valu_active_frac'])} | {fmt(iss['issue_active_frac'])} | {fmt(iss['wait_frac'])} | "
                    f"{fmt(iss['simd_frac'])} | {fmt(iss['chip_valu_frac'])} | {fmt(iss['f64_share'])} | "
                    f"{fmt(iss['kernel_us_from_counters'], 1)} | {fmt(rp, 1)} | {fmt(ratio, 2)} |")
    return "\n".join(rows)


def main():
    with open(sys.argv[1]) as fh:
        d = json.load(fh)
    shas = [(e.get("traffic_detail") or {}).get("lib_sha16") for _, e in entries(d)]
    sha = next((s for s in shas if s), None)
    print(f"library {sha}; headline value {d['value']:.4g} env-steps/s, {d['ms_per_step'] * 1e3:.2f} µs/step wall\n")
    print(roofline_table(d))
    print()
    print(issue_table(d))


if __name__ == "__main__":
    main()
