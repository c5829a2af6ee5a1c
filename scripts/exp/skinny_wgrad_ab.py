"""A/B of the learner's skinny weight gradients dW = dYᵀ X with K = 65 536 rows (one PPO minibatch of the
16 x 8192 rollout) and one small side: the 13-input layers (actor trunk 13 -> 512, critic 13 -> 256) and the
one- / four-output heads.  rocprof of the update (profiles/r05/learn/) puts three such hipBLASLt kernels at
136 / 64 / 32 us each, far above the ~30 us it takes to read dY once.  Prints one JSON line per (shape, form):
median GPU us over 50 calls and the max relative difference from the f64 product.
    python scripts/exp/skinny_wgrad_ab.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from ouzelum_amd.learners.fused import splitk_wgrad  # noqa: E402

dev = torch.device("cuda", 0)
K = 65536


def splitk(dy, x, s):
    k, n = dy.shape
    return torch.bmm(dy.view(s, k // s, n).transpose(1, 2), x.view(s, k // s, x.shape[1])).sum(0)


def forms(n_out, n_in):
    f = {
        "splitk_wgrad (current)": lambda dy, x: splitk_wgrad(dy, x),
        "dy.t().mm(x)": lambda dy, x: dy.t().mm(x),
        "x.t().mm(dy).t()": lambda dy, x: x.t().mm(dy).t(),
    }
    for s in (4, 8, 16, 64, 128, 256):
        f[f"splitk s={s}"] = (lambda s: lambda dy, x: splitk(dy, x, s))(s)
        f[f"splitk_T s={s}"] = (lambda s: lambda dy, x: splitk(x, dy, s).t())(s)
    return f


def main():
    torch.manual_seed(0)
    for n_out, n_in in ((512, 13), (256, 13), (1, 256), (4, 128), (512, 256), (256, 256)):
        dy = torch.randn(K, n_out, device=dev)
        x = torch.randn(K, n_in, device=dev)
        ref = dy.double().t().mm(x.double())
        for name, fn in forms(n_out, n_in).items():
            try:
                out = fn(dy, x)
            except RuntimeError as e:
                print(json.dumps({"n_out": n_out, "n_in": n_in, "form": name, "error": str(e)[:80]}), flush=True)
                continue
            err = float(((out.double() - ref).abs().max() / ref.abs().max()))
            for _ in range(5):
                fn(dy, x)
            torch.cuda.synchronize()
            ts = []
            for _ in range(50):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                fn(dy, x)
                e.record()
                e.synchronize()
                ts.append(s.elapsed_time(e) * 1e3)
            ts.sort()
            print(json.dumps({"n_out": n_out, "n_in": n_in, "form": name, "us": round(ts[len(ts) // 2], 1),
                              "rel_err": err}), flush=True)


if __name__ == "__main__":
    main()
