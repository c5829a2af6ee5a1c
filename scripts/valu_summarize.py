"""Issue-bound summary of one kernel from scripts/gpu_valu.sh's two PMC passes.

    python valu_summarize.py OUTDIR TAG TASK N MODE   -> OUTDIR/valu_TAG_MODE_TASK_N_summary.json

Counter units (MI355X_MICROARCH.md §rocprofv3 / the counter descriptions of `rocprofv3 -L` on gfx950):
SQ_WAVE_CYCLES, SQ_ACTIVE_INST_*, SQ_WAIT_* are wave quad-cycles summed over the waves; SQ_WAIT_ANY +
SQ_WAIT_INST_ANY + SQ_ACTIVE_INST_ANY ~= SQ_WAVE_CYCLES; GRBM_GUI_ACTIVE is GPU-busy cycles summed over the 8
XCDs.  Derived, per dispatch of the kernel (averaged over its dispatches):
  clock_ghz          GRBM_GUI_ACTIVE / 8 / the dispatch's duration (kernel trace of the same pass; reads high on
                     dispatches shorter than ~0.3 ms, the guide's DVFS note)
  wave_cycles        one wave's lifetime in shader cycles, SQ_WAVE_CYCLES * 4 / SQ_WAVES; kernel_cycles GRBM / 8
  wave_us            one wave's lifetime, SQ_WAVE_CYCLES * 4 / SQ_WAVES / clock
  valu_active_frac   SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES: share of a wave's life its VALU instructions occupy
  issue_active_frac  SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES (any instruction issuing); wait_frac (s_waitcnt /
                     barrier parked) and inst_stall_frac (issue stalls) make up the rest
  valu_issue_frac    SQ_INSTS_VALU * 4 cycles / wave lifetime: against ONE wave's issue floor (an instruction
                     every 4 cycles, the row 'vector-instruction ISSUE cost' of the guide) -- the bound of the
                     latency regime, where each SIMD holds one wave
  chip_valu_frac     SQ_ACTIVE_INST_VALU * 4 / (1024 SIMDs * kernel cycles): the chip's VALU time in use
  simd_frac          SQ_WAVE_CYCLES * 4 / (1024 * kernel cycles): SIMD-time occupied by waves (<= waves per SIMD)
  f64_share          f64 FMA + MUL + ADD + TRANS instructions / SQ_INSTS_VALU
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summarize import lib_sha16  # noqa: E402

N_SIMDS = 256 * 4
N_XCD = 8


def rows(base, k, kname):
    """{dispatch: {counter: value}} and {dispatch: duration_ns} of the kernel in pass k."""
    vals, dur = defaultdict(dict), {}
    for f in glob.glob(f"{base}_p{k}/**/*counter_collection.csv", recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if kname not in r.get("Kernel_Name", ""):
                    continue
                d = int(r["Dispatch_Id"])
                vals[d][r["Counter_Name"]] = vals[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
                dur[d] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return vals, dur


def avg(dicts, key):
    v = [d[key] for d in dicts if key in d]
    return sum(v) / len(v) if v else None


def main():
    out, tag, task, n, mode = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]), sys.argv[5]
    kname = "quad_rollout_kernel<" if mode == "rollout" else "quad_step_kernel<"
    base = os.path.join(out, f"valu_{tag}_{mode}_{task}_{n}")
    v1, d1 = rows(base, 1, kname)
    v2, d2 = rows(base, 2, kname)
    if not v1 or not v2:
        raise SystemExit(f"no {kname} dispatches in {base}_p1/_p2")
    p1, p2 = list(v1.values()), list(v2.values())
    c = {k: avg(p1, k) for k in ("SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_INSTS_VALU",
                                 "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY",
                                 "GRBM_GUI_ACTIVE", "GRBM_COUNT")}
    c2 = {k: avg(p2, k) for k in ("SQ_WAVES", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64",
                                  "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_TRANS_F64", "SQ_INSTS_VALU_TRANS_F32",
                                  "SQ_INSTS_SALU", "SQ_INSTS_VMEM", "GRBM_GUI_ACTIVE")}
    dur_us = sum(d1.values()) / len(d1) / 1e3
    kcyc = c["GRBM_GUI_ACTIVE"] / N_XCD
    clock = kcyc / (dur_us * 1e3)
    waves = c["SQ_WAVES"]
    wc = c["SQ_WAVE_CYCLES"]
    steps = 1
    if mode == "rollout":   # kernel_driver.py's default launch length (bench.evidence_launch_steps)
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from bench import evidence_launch_steps
        steps = int(sys.argv[6]) if len(sys.argv) > 6 else evidence_launch_steps(n)
    f64 = sum(c2[k] or 0.0 for k in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64",
                                     "SQ_INSTS_VALU_TRANS_F64"))
    res = {"task": task, "num_envs": n, "mode": mode, "kernel": kname.rstrip("<"), "steps_per_launch": steps,
           "dispatches": [len(v1), len(v2)], "lib_sha16": lib_sha16(), "counters_pass1": c, "counters_pass2": c2,
           "kernel_us_pmc_pass": round(dur_us, 3), "clock_ghz": round(clock, 3),
           "wave_cycles": round(wc * 4 / waves, 1), "kernel_cycles": round(kcyc, 1),
           "wave_us": round(wc * 4 / waves / (clock * 1e3), 3),
           "valu_active_frac": round(c["SQ_ACTIVE_INST_VALU"] / wc, 4),
           "issue_active_frac": round(c["SQ_ACTIVE_INST_ANY"] / wc, 4),
           "wait_frac": round(c["SQ_WAIT_ANY"] / wc, 4), "inst_stall_frac": round(c["SQ_WAIT_INST_ANY"] / wc, 4),
           "valu_issue_frac": round(c["SQ_INSTS_VALU"] * 4 / (wc * 4 / waves * waves), 4),
           "chip_valu_frac": round(c["SQ_ACTIVE_INST_VALU"] * 4 / (N_SIMDS * kcyc), 4),
           "simd_frac": round(wc * 4 / (N_SIMDS * kcyc), 4),
           "valu_insts_per_wave_step": round(c["SQ_INSTS_VALU"] / waves / steps, 1),
           "valu_cycles_per_inst": round(c["SQ_ACTIVE_INST_VALU"] * 4 / c["SQ_INSTS_VALU"], 3),
           "f64_share": round(f64 / c["SQ_INSTS_VALU"], 4) if c["SQ_INSTS_VALU"] else None,
           "salu_per_valu": round((c2["SQ_INSTS_SALU"] or 0) / c["SQ_INSTS_VALU"], 4)}
    with open(base + "_summary.json", "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps({k: v for k, v in res.items() if not k.startswith("counters")}))


if __name__ == "__main__":
    main()
