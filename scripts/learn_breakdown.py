"""Per-iteration kernel-time breakdown of the RPO-LSTM learner from a rocprofv3 --kernel-trace --stats summary of
scripts/bench_learner.py, with the update's GEMM FLOPs priced against the f32 MFMA peak.

    python scripts/learn_breakdown.py profiles/r05/learn/learn_QuadFault_8192_kernel_stats.csv 10 8192 \
        > profiles/r05/learn/learn_breakdown_QuadFault_8192.json

FLOPs (RPO-LSTM/model.py:11-84 shapes, models.py here): actor 13-512-256 trunk, LSTM(256, 128) (input and
recurrent projections, 4H = 512), 128-4 mean head; critic 13-256-256-1.  Forward 2 FLOP per multiply-add,
backward 4 (input and weight gradients); the update is 4 epochs over T x N samples (PPOLearner defaults), plus
the critic's value pass over the rollout and the rollout's own policy forward (T steps x N envs).
"""
import csv
import json
import sys

PEAK_F32_MFMA_TF = 157.3          # MI355X_MICROARCH.md: f32 matrix = f32 vector peak, exact f32
T_STEPS, EPOCHS = 16, 4
ACTOR_MACS = 13 * 512 + 512 * 256 + 256 * 512 + 128 * 512 + 128 * 4
CRITIC_MACS = 13 * 256 + 256 * 256 + 256 * 1


def category(name):
    if name.startswith("Cijk_"):
        return "gemm (hipBLASLt)"
    if "copyBuffer" in name or "fillBuffer" in name:
        return "runtime copy / fill"
    if "lstm_cell" in name:
        return "lstm cell (HIP)"
    if "lstm_seq" in name:
        return "lstm recurrence, one launch per direction (HIP, f32 MFMA)"
    if any(k in name for k in ("policy_loss_kernel", "value_loss_kernel", "loss_finish_kernel", "adv_moments_kernel",
                                "tanh_bwd_colsum_kernel", "colsum_finish_kernel")):
        return "PPO losses + trunk tanh'/bias (HIP)"
    if "linear_tanh_smallk" in name:
        return "trunks' first layer + tanh (HIP, one pass)"
    if "adam_step_kernel" in name or "adam_sqnorm_kernel" in name:
        return "clipped Adam (HIP, two launches)"
    if "FusedOptimizer" in name or "multi_tensor_apply" in name:
        return "fused Adam / grad-norm (multi-tensor)"
    if "reduce_kernel" in name:
        return "reduction (bias grads, split-K sums, norms, means)"
    if "ouz::" in name or "ouz_" in name or "pomdp_obs_kernel" in name or "gae_kernel" in name:
        return "env + learner HIP kernels"
    if "elementwise" in name or "index" in name or "Fill" in name:
        return "elementwise / gather"
    return "other"


def main():
    path, iters, n = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    rows = list(csv.DictReader(open(path)))
    cats, tops = {}, []
    for r in rows:
        ms = float(r["TotalDurationNs"]) / 1e6 / iters
        c = category(r["Name"])
        d = cats.setdefault(c, {"ms_per_iter": 0.0, "launches_per_iter": 0.0})
        d["ms_per_iter"] += ms
        d["launches_per_iter"] += int(r["Calls"]) / iters
        tops.append((ms, int(r["Calls"]) / iters, float(r["AverageNs"]) / 1e3, r["Name"][:96]))
    total = sum(d["ms_per_iter"] for d in cats.values())
    samples = T_STEPS * n
    upd = EPOCHS * samples * 6 * (ACTOR_MACS + CRITIC_MACS) + samples * 2 * CRITIC_MACS
    roll = samples * 2 * ACTOR_MACS
    gemm_ms = cats.get("gemm (hipBLASLt)", {}).get("ms_per_iter", 0.0)
    out = {
        "source": path, "iterations_profiled": iters, "num_envs": n, "rollout_steps": T_STEPS, "epochs": EPOCHS,
        "kernel_ms_per_iter": round(total, 3),
        "by_category": {k: {"ms_per_iter": round(v["ms_per_iter"], 3), "share": round(v["ms_per_iter"] / total, 3),
                            "launches_per_iter": round(v["launches_per_iter"], 1)}
                        for k, v in sorted(cats.items(), key=lambda kv: -kv[1]["ms_per_iter"])},
        "gemm_flop_per_iter": {"update": upd, "rollout_policy": roll},
        "gemm_tflops_achieved": round((upd + roll) / (gemm_ms * 1e-3) / 1e12, 1) if gemm_ms else None,
        "gemm_frac_of_f32_mfma_peak": round((upd + roll) / (gemm_ms * 1e-3) / 1e12 / PEAK_F32_MFMA_TF, 3)
        if gemm_ms else None,
        "update_gemm_floor_ms": round(upd / (PEAK_F32_MFMA_TF * 1e12) * 1e3, 2),
        "top_kernels": [{"ms_per_iter": round(m, 3), "launches_per_iter": c, "avg_us": round(a, 1), "name": nm}
                        for m, c, a, nm in sorted(tops, reverse=True)[:15]],
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
