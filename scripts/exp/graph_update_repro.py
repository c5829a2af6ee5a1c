"""Torch-only repro matrix for the dropped hipGraph capture of the learner update.

One "update" = E epochs x M minibatches of (gather rows, MLP forward, MSE loss, backward, clip_grad_norm_,
optimizer step), the PPO update's op mix without this repo's kernels.  A graphed learner (whole update
captured once, replayed per update with fresh data copied into static buffers) is compared bitwise with an
eager learner from the same initial state over R updates, and every replay is checked for determinism
(replayed twice from the same snapshot of parameters / optimizer state).

    python scripts/exp/graph_update_repro.py --variant sgd [--churn] [--env K=V ...]

--variant  sgd: SGD, zero_grad(set_to_none=True) in the capture; sgd_zero: grads pre-allocated and zeroed
           in the capture; adam: Adam(capturable=True)
--churn    eager allocation churn between replays (new data tensors per update, freed the next one, the
           way the rollout / eager code allocates between two updates); without it every tensor used
           after the capture is allocated before it
--env      environment variables set before torch is imported (e.g. HIPBLASLT_WORKSPACE_SIZE=0,
           TORCH_BLAS_PREFER_HIPBLASLT=0)
"""
import argparse
import json
import os

ap = argparse.ArgumentParser()
ap.add_argument("--variant", default="sgd", choices=["sgd", "sgd_zero", "adam"])
ap.add_argument("--churn", action="store_true")
ap.add_argument("--env", nargs="*", default=[])
ap.add_argument("--updates", type=int, default=10)
a = ap.parse_args()
for kv in a.env:
    k, v = kv.split("=", 1)
    os.environ[k] = v

import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

dev = torch.device("cuda", 0)
N, T, D_IN, D_OUT, H = 4096, 16, 13, 4, 256
E, M = 4, 2


def model(seed):
    torch.manual_seed(seed)
    return nn.Sequential(nn.Linear(D_IN, H), nn.Tanh(), nn.Linear(H, H), nn.Tanh(), nn.Linear(H, D_OUT)).to(dev)


def data(r, out=None):
    g = torch.Generator(device=dev).manual_seed(1000 + r)
    if out is None:
        out = (torch.empty((T * N, D_IN), device=dev), torch.empty((T * N, D_OUT), device=dev))
    out[0].normal_(generator=g)
    out[1].normal_(generator=g)
    return out


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


def make_opt(net):
    if a.variant == "adam":
        return torch.optim.Adam(net.parameters(), lr=2.6e-3, eps=1e-5, capturable=True)
    return torch.optim.SGD(net.parameters(), lr=1e-2)


def state_tensors(net, opt):
    ts = [p.data for p in net.parameters()]
    for p in net.parameters():
        for k in sorted(opt.state.get(p, {})):
            v = opt.state[p][k]
            if torch.is_tensor(v):
                ts.append(v)
    return ts


def flat(net):
    return torch.cat([p.detach().reshape(-1) for p in net.parameters()])


def main():
    set_to_none = a.variant != "sgd_zero"
    eager, graphed = model(0), model(0)
    opt_e, opt_g = make_opt(eager), make_opt(graphed)
    Xs, Ys = data(0)
    if not set_to_none:
        for net in (eager, graphed):
            for p in net.parameters():
                p.grad = torch.zeros_like(p)
    side = torch.cuda.Stream(device=dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        for _ in range(3):
            update(graphed, opt_g, Xs, Ys, set_to_none)
    torch.cuda.current_stream(dev).wait_stream(side)
    # both learners start from the warmed-up state (copied in place into the eager learner)
    update(eager, opt_e, Xs, Ys, set_to_none)   # creates the eager optimizer state
    with torch.no_grad():
        for d, s in zip(state_tensors(eager, opt_e), state_tensors(graphed, opt_g)):
            d.copy_(s)
    snap = [t.clone() for t in state_tensors(graphed, opt_g)]   # determinism snapshot, allocated up front
    pre = [data(r) for r in range(a.updates)] if not a.churn else None
    res_a = torch.empty_like(flat(graphed))
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        update(graphed, opt_g, Xs, Ys, set_to_none)
    torch.cuda.synchronize(dev)
    diffs, det = [], []
    for r in range(a.updates):
        X, Y = data(r) if a.churn else pre[r]
        update(eager, opt_e, X, Y, set_to_none)
        Xs.copy_(X)
        Ys.copy_(Y)
        with torch.no_grad():
            for s, t in zip(snap, state_tensors(graphed, opt_g)):
                s.copy_(t)
        graph.replay()
        res_a.copy_(flat(graphed))
        with torch.no_grad():
            for s, t in zip(snap, state_tensors(graphed, opt_g)):
                t.copy_(s)
        graph.replay()
        det.append(bool(torch.equal(res_a, flat(graphed))))
        diffs.append(float((flat(graphed) - flat(eager)).abs().max()))
        if a.churn:   # allocations of assorted sizes between updates, freed again
            junk = [torch.empty(int(s), device=dev) for s in (1 << 12, 3 << 16, 1 << 20, 5 << 14)]
            del junk
    torch.cuda.synchronize(dev)
    print(json.dumps({"variant": a.variant, "churn": a.churn, "env": a.env,
                      "max_abs_param_diff_per_update": [float(f"{d:.3g}") for d in diffs],
                      "replay_deterministic": det}), flush=True)


if __name__ == "__main__":
    main()
