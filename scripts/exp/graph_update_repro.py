"""Torch-only repro matrix for the dropped hipGraph capture of the learner update.

One "update" = E epochs x M minibatches of (gather rows, MLP forward, MSE loss, backward, clip_grad_norm_,
optimizer step), the PPO update's op mix without this repo's kernels.  A graphed learner (whole update
captured once, replayed per update with fresh data copied into static buffers) is compared bitwise with an
eager learner from the same initial state over R updates.  Variants isolate the suspects:

  sgd_none     SGD, zero_grad(set_to_none=True) inside the capture
  sgd_zero     SGD, grads pre-allocated, zero_grad(set_to_none=False) (memset nodes) inside the capture
  adam_cap     Adam(capturable=True)
  sgd_restore  sgd_none, but the warm-up's parameter changes undone by copy_ into the same tensors
  sgd_noresto  sgd_none, warm-up changes NOT undone (the learner starts from the warmed-up params)

Prints one JSON line per variant: per-update max |param_graph - param_eager| and whether the graph replays
are deterministic (the same update replayed twice from the same state).
"""
import copy
import json
import sys

import torch
import torch.nn as nn

dev = torch.device("cuda", 0)
N, T, D_IN, D_OUT, H = 4096, 16, 13, 4, 256
E, M, R = 4, 2, 6


def model(seed):
    torch.manual_seed(seed)
    return nn.Sequential(nn.Linear(D_IN, H), nn.Tanh(), nn.Linear(H, H), nn.Tanh(), nn.Linear(H, D_OUT)).to(dev)


def data(r):
    g = torch.Generator(device=dev).manual_seed(1000 + r)
    return (torch.randn((T * N, D_IN), device=dev, generator=g), torch.randn((T * N, D_OUT), device=dev, generator=g))


# fixed minibatch index lists (deterministic permutations)
g0 = torch.Generator(device=dev).manual_seed(7)
IDX = [torch.randperm(T * N, device=dev, generator=g0).reshape(M, -1) for _ in range(E)]


def update(net, opt, X, Y, set_to_none):
    loss = None
    for e in range(E):
        for m in range(M):
            idx = IDX[e][m]
            out = net(X[idx])
            loss = ((out - Y[idx]) ** 2).mean()
            opt.zero_grad(set_to_none=set_to_none)
            loss.backward()
            nn.utils.clip_grad_norm_(net.parameters(), 1.0)
            opt.step()
    return loss.detach()


def make_opt(net, kind):
    if kind == "adam":
        return torch.optim.Adam(net.parameters(), lr=2.6e-3, eps=1e-5, capturable=True)
    return torch.optim.SGD(net.parameters(), lr=1e-2)


def flat(net):
    return torch.cat([p.detach().reshape(-1) for p in net.parameters()])


def run(variant):
    kind = "adam" if variant.startswith("adam") else "sgd"
    set_to_none = variant != "sgd_zero"
    eager = model(0)
    graphed = model(0)
    opt_e, opt_g = make_opt(eager, kind), make_opt(graphed, kind)
    Xs, Ys = data(0)
    Xs, Ys = Xs.clone(), Ys.clone()
    init_params = [p.detach().clone() for p in graphed.parameters()]
    if not set_to_none:
        for p in graphed.parameters():
            p.grad = torch.zeros_like(p)
        for p in eager.parameters():
            p.grad = torch.zeros_like(p)
    side = torch.cuda.Stream(device=dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        for _ in range(3):
            update(graphed, opt_g, Xs, Ys, set_to_none)
    torch.cuda.current_stream(dev).wait_stream(side)
    if variant != "sgd_noresto":
        with torch.no_grad():
            for p, p0 in zip(graphed.parameters(), init_params):
                p.copy_(p0)
        if kind == "adam":   # undo the warm-up's optimizer state in place (the graph holds these tensors)
            for st in opt_g.state.values():
                for k, v in st.items():
                    if torch.is_tensor(v):
                        v.zero_()
    else:
        eager.load_state_dict(graphed.state_dict())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        out = update(graphed, opt_g, Xs, Ys, set_to_none)
    # the capture does not execute: the graphed learner is still at its initial (or warmed-up) state
    diffs, det = [], []
    for r in range(R):
        X, Y = data(r)
        update(eager, opt_e, X, Y, set_to_none)
        Xs.copy_(X)
        Ys.copy_(Y)
        # determinism probe: replay, snapshot, restore, replay again
        snap_p = [p.detach().clone() for p in graphed.parameters()]
        snap_s = copy.deepcopy({k: {kk: (vv.clone() if torch.is_tensor(vv) else vv) for kk, vv in v.items()}
                                for k, v in opt_g.state.items()})
        graph.replay()
        a = flat(graphed).clone()
        with torch.no_grad():
            for p, s in zip(graphed.parameters(), snap_p):
                p.copy_(s)
            for k, v in opt_g.state.items():
                for kk, vv in v.items():
                    if torch.is_tensor(vv):
                        vv.copy_(snap_s[k][kk])
        graph.replay()
        b = flat(graphed)
        det.append(bool(torch.equal(a, b)))
        diffs.append(float((flat(graphed) - flat(eager)).abs().max()))
    torch.cuda.synchronize(dev)
    return {"variant": variant, "max_abs_param_diff_per_update": diffs, "replay_deterministic": det,
            "loss_graph": float(out)}


if __name__ == "__main__":
    for v in (sys.argv[1:] or ["sgd_none", "sgd_zero", "adam_cap", "sgd_noresto"]):
        try:
            print(json.dumps(run(v)), flush=True)
        except Exception as exc:  # noqa: BLE001
            print(json.dumps({"variant": v, "error": repr(exc)[:400]}), flush=True)
