"""A fixed workload of the fused LSTM sequence kernels for rocprofv3 PMC passes (round 6): config D's update shape,
T = 16, B = 4096, H = 128, forward + BPTT through fused.LSTMSequence, ``--iters`` times.
    python scripts/exp/lstm_seq_probe.py [--iters 20] [--seq 1]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--T", type=int, default=16)
ap.add_argument("--B", type=int, default=4096)
ap.add_argument("--seq", default="1")
a = ap.parse_args()
os.environ["OUZ_LSTM_SEQ"] = a.seq
from ouzelum_amd.learners import fused as F  # noqa: E402

g = torch.Generator(device="cuda").manual_seed(0)
T, B, H = a.T, a.B, 128
xp = torch.randn((T, B, 4 * H), device="cuda", generator=g).requires_grad_(True)
h0 = torch.randn((B, H), device="cuda", generator=g)
c0 = torch.randn((B, H), device="cuda", generator=g)
keep = (torch.rand((T, B), device="cuda", generator=g) > 0.1).float()
w = (torch.randn((4 * H, H), device="cuda", generator=g) * H ** -0.5).requires_grad_(True)
up = torch.randn((T, B, H), device="cuda", generator=g)
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for it in range(a.iters + 3):
    if it == 3:
        s.record()
    hid, hT, cT = F.LSTMSequence.apply(xp, h0, c0, keep, w)
    (hid * up).sum().backward()
e.record()
torch.cuda.synchronize()
print(f"seq={a.seq} T={T} B={B}: {s.elapsed_time(e) / a.iters * 1e3:.1f} us per forward + backward")
