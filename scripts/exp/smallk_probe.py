"""The trunks' first layer (K = 13) + tanh: ouz_linear_tanh_small_k against hipBLASLt's GEMM + torch's tanh, GPU
time per call at the learner's shapes (round 6).   python scripts/exp/smallk_probe.py [--iters 50]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from ouzelum_amd.learners.fused import linear_tanh_small_k  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=50)
a = ap.parse_args()
for rows, cols in ((8192, 512), (8192, 256), (65536, 512), (65536, 256), (131072, 256)):
    lin = torch.nn.Linear(13, cols).cuda()
    x = torch.randn(rows, 13, device="cuda")
    res = {"rows": rows, "k": 13, "cols": cols}
    with torch.no_grad():
        for name, fn in (("small_k", lambda: linear_tanh_small_k(x, lin.weight, lin.bias)),
                         ("gemm_tanh", lambda: torch.tanh_(torch.addmm(lin.bias, x, lin.weight.t())))):
            for _ in range(5):
                fn()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.iters):
                fn()
            e.record()
            torch.cuda.synchronize()
            res[name + "_us"] = round(s.elapsed_time(e) / a.iters * 1e3, 2)
    print(json.dumps(res), flush=True)
