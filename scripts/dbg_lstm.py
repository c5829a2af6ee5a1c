import sys
import torch
sys.path.insert(0, ".")
from ouzelum_amd.learners.fused import LSTMSequence
torch.manual_seed(0)
T, B, H = 4, 8, 4
dev = "cuda"
x_proj = torch.randn(T, B, 4 * H, device=dev, requires_grad=True)
h0 = torch.randn(B, H, device=dev); c0 = torch.randn(B, H, device=dev)
keep = (torch.rand(T, B, device=dev) > 0.3).float()
W = torch.randn(4 * H, H, device=dev, requires_grad=True)
wout = torch.randn(T, B, H, device=dev)
def ref():
    h, c = h0, c0; outs = []
    for t in range(T):
        hm = keep[t, :, None] * h; cm = keep[t, :, None] * c
        g = x_proj[t] + hm @ W.t()
        i, f, gg, o = g.chunk(4, 1)
        i, f, gg, o = i.sigmoid(), f.sigmoid(), gg.tanh(), o.sigmoid()
        c = f * cm + i * gg; h = o * c.tanh(); outs.append(h)
    return torch.stack(outs), h, c
for name, fn in (("ref", ref), ("fused", lambda: LSTMSequence.apply(x_proj, h0, c0, keep, W))):
    x_proj.grad = None; W.grad = None
    hid, hT, cT = fn()
    L = (hid * wout).sum() + hT.sum() * 0.5 + cT.sum() * 0.25
    L.backward()
    print(name, "hid", hid[:, 0, 0].tolist())
    print(name, "gx per t", [float(x_proj.grad[t].abs().sum()) for t in range(T)])
    print(name, "gW", float(W.grad.abs().sum()))
