"""Launch-count trims of the learner's data movement (round 6), GPU µs per call at config D's sizes (N = 8192, T = 16):
the rollout's five per-step storage copies as separate copies against one torch._foreach_copy_, and a minibatch's
seven per-sample gathers (x[mb_inds]) against index_select and against one index_select of the four per-row scalars
stacked.   python scripts/exp/copy_gather_probe.py"""
import json
import torch

N, T, it = 8192, 16, 200
dev = torch.device("cuda")
ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731


def timed(fn):
    for _ in range(10):
        fn()
    s, e = ev(), ev()
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e) / it * 1e3, 2)


obs = torch.zeros((T, N, 13), device=dev); pomdps = torch.zeros_like(obs); dones = torch.zeros((T, N), device=dev)
actions = torch.zeros((T, N, 4), device=dev); logprobs = torch.zeros((T, N), device=dev)
o, p, d, a, lp = (torch.randn(N, 13, device=dev), torch.randn(N, 13, device=dev), torch.rand(N, device=dev),
                  torch.randn(N, 4, device=dev), torch.randn(N, device=dev))


def sep():
    pomdps[3] = p; obs[3] = o; dones[3] = d; actions[3] = a; logprobs[3] = lp


def fe():
    torch._foreach_copy_([pomdps[3], obs[3], dones[3], actions[3], logprobs[3]], [p, o, d, a, lp])


print(json.dumps({"rollout_copies_separate_us": timed(sep), "rollout_copies_foreach_us": timed(fe)}))
B = T * N
b13a, b13b, b4 = torch.randn(B, 13, device=dev), torch.randn(B, 13, device=dev), torch.randn(B, 4, device=dev)
s1 = [torch.randn(B, device=dev) for _ in range(4)]
stack = torch.stack(s1)
idx = torch.randperm(B, device=dev)[: B // 2]


def adv():
    return b13a[idx], b13b[idx], b4[idx], s1[0][idx], s1[1][idx], s1[2][idx], s1[3][idx]


def isel():
    return tuple(torch.index_select(x, 0, idx) for x in (b13a, b13b, b4, *s1))


def stacked():
    return (torch.index_select(b13a, 0, idx), torch.index_select(b13b, 0, idx), torch.index_select(b4, 0, idx),
            torch.index_select(stack, 1, idx))


print(json.dumps({"gathers_advanced_index_us": timed(adv), "gathers_index_select_us": timed(isel),
                  "gathers_stacked_scalars_us": timed(stacked)}))
