"""GPU-side building blocks of the recurrent learner (HIP + hipBLASLt), with autograd.

* ``LSTMSequence``: the whole done-masked recurrence of ``RPO-LSTM/model.py:34-50`` over T
  steps.  Per step one hipBLASLt GEMM (h W_hh^T added onto the precomputed input projection)
  and ONE fused HIP cell kernel (``ouz_lstm_cell_fwd``); BPTT is the mirror image
  (``ouz_lstm_cell_bwd`` + one GEMM per step) and dW_hh is one split-K product over all
  T·B rows.  torch's per-step nn.LSTM costs ~10 element-wise launches forward and ~20
  backward per step.
* ``splitk_wgrad`` / ``SplitKLinear``: weight gradients dW = dYᵀ X with K = T·B rows
  (32 768 at the reference's 16 x 4096 minibatch halves) and a small output (512 x 256):
  a plain GEMM puts 16 output tiles on 256 CUs; splitting K into S slabs and summing
  gives 16·S workgroups.
"""
import os

import torch

from .. import _lib as L

_INPLACE_GATES = os.environ.get("OUZ_LSTM_INPLACE_GATES", "1") != "0"


def _splits(k, n_out_tiles):
    """Number of K slabs: enough workgroups to cover the chip, slabs of >= 256 rows."""
    for s in (32, 16, 8, 4, 2):
        if k % s == 0 and k // s >= 256 and n_out_tiles * s <= 1024:
            return s
    return 1


def splitk_wgrad(dy, x):
    """dy (K, N), x (K, M) -> dyᵀ x (N, M) with K split into slabs (one batched GEMM + a sum)."""
    k, n = dy.shape
    m = x.shape[1]
    s = _splits(k, max(1, (n // 64) * (m // 64)))
    if s == 1:
        return dy.t().mm(x)
    return torch.bmm(dy.view(s, k // s, n).transpose(1, 2), x.view(s, k // s, m)).sum(0)


class SplitKLinear(torch.autograd.Function):
    """y = x Wᵀ + b with the split-K weight gradient."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        ctx.save_for_backward(x, weight)
        ctx.has_bias = bias is not None
        return torch.addmm(bias, x, weight.t()) if bias is not None else x.mm(weight.t())

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        dy = dy.contiguous()
        dx = dy.mm(weight) if ctx.needs_input_grad[0] else None
        dw = splitk_wgrad(dy, x.contiguous()) if ctx.needs_input_grad[1] else None
        db = dy.sum(0) if ctx.has_bias and ctx.needs_input_grad[2] else None
        return dx, dw, db


def linear(x, layer, min_rows=8192):
    """nn.Linear forward; rows >= min_rows on a GPU take the split-K weight gradient."""
    if x.is_cuda and x.dim() == 2 and x.shape[0] >= min_rows and torch.is_grad_enabled():
        return SplitKLinear.apply(x, layer.weight, layer.bias)
    return torch.nn.functional.linear(x, layer.weight, layer.bias)


def run_mlp(seq, x):
    """Forward through an nn.Sequential of Linear / activation modules using ``linear``."""
    for m in seq:
        x = linear(x, m) if isinstance(m, torch.nn.Linear) else m(x)
    return x


def _p(t):
    return None if t is None else t.data_ptr()


class LSTMSequence(torch.autograd.Function):
    """(x_proj (T,B,4H), h0 (B,H), c0 (B,H), keep (T,B), W_hh (4H,H)) -> (hidden (T,B,H), h_T, c_T).
    keep[t] = 1 - done[t] zeroes the carry entering step t (model.py:42-46)."""

    @staticmethod
    def forward(ctx, x_proj, h0, c0, keep, w_hh):
        T, B, G4 = x_proj.shape
        H = G4 // 4
        dev = x_proj.device
        stream = L.stream_ptr(dev)
        x_proj = x_proj.contiguous()
        keep = keep.contiguous().float()
        act = torch.empty((T, B, G4), device=dev)
        c_all = torch.empty((T, B, H), device=dev)
        hid = torch.empty((T, B, H), device=dev)
        hm = torch.empty((T + 1, B, H), device=dev)       # masked h entering each step (+1 scratch)
        cm = torch.empty((T + 1, B, H), device=dev)       # masked c entering each step
        torch.mul(h0, keep[0].unsqueeze(1), out=hm[0])
        torch.mul(c0, keep[0].unsqueeze(1), out=cm[0])
        inplace = _INPLACE_GATES
        gates = None if inplace else torch.empty((B, G4), device=dev)
        w_t = w_hh.t()
        for t in range(T):
            if inplace:
                # the recurrent product accumulates onto the step's input projection in place (beta = 1, C = D):
                # addmm with out= a separate buffer first copies the (B, 4H) projection into it, one runtime
                # copy launch per step.  x_proj is this function's own temporary (SplitKLinear / addmm output)
                # and is not saved for the backward pass.
                gates = x_proj[t]
                torch.addmm(gates, hm[t], w_t, out=gates)
            else:
                torch.addmm(x_proj[t], hm[t], w_t, out=gates)
            kn = keep[t + 1] if t + 1 < T else None
            L.check(L.lib.ouz_lstm_cell_fwd(gates.data_ptr(), cm[t].data_ptr(), _p(kn), act[t].data_ptr(),
                                            c_all[t].data_ptr(), hid[t].data_ptr(), hm[t + 1].data_ptr(),
                                            cm[t + 1].data_ptr(), B, H, stream), "ouz_lstm_cell_fwd")
        ctx.save_for_backward(act, c_all, cm, hm, keep, w_hh)
        return hid, hid[T - 1].clone(), c_all[T - 1].clone()

    @staticmethod
    def backward(ctx, dhid, dhT, dcT):
        act, c_all, cm, hm, keep, w_hh = ctx.saved_tensors
        T, B, G4 = act.shape
        H = G4 // 4
        dev = act.device
        stream = L.stream_ptr(dev)
        dhid = torch.zeros((T, B, H), device=dev) if dhid is None else dhid.contiguous()
        # keep the contiguous copies alive until the kernels have run (expanded grads of a sum are
        # stride-0 views; a temporary's block would be handed to the next allocation)
        dhT = dhT.contiguous() if dhT is not None else None
        dcT = dcT.contiguous() if dcT is not None else None
        dgates = torch.empty((T, B, G4), device=dev)
        G = torch.empty((B, H), device=dev)
        dc = torch.empty((B, H), device=dev)
        for t in range(T - 1, -1, -1):
            if t == T - 1:
                g_ptr, dcn = _p(dhT), _p(dcT)
                kn = None
            else:
                torch.mm(dgates[t + 1], w_hh, out=G)
                g_ptr, dcn, kn = G.data_ptr(), dc.data_ptr(), keep[t + 1].data_ptr()
            # dc is read (dc_next) and written (dc_prev) element-wise by the same thread: in place is safe
            L.check(L.lib.ouz_lstm_cell_bwd(act[t].data_ptr(), c_all[t].data_ptr(), cm[t].data_ptr(),
                                            dhid[t].data_ptr(), g_ptr, dcn, kn, dgates[t].data_ptr(),
                                            dc.data_ptr(), B, H, stream), "ouz_lstm_cell_bwd")
        d_w = splitk_wgrad(dgates.view(T * B, G4), hm[:T].reshape(T * B, H)) if ctx.needs_input_grad[4] else None
        k0 = keep[0].unsqueeze(1)
        dh0 = dgates[0].mm(w_hh) * k0 if ctx.needs_input_grad[1] else None
        dc0 = dc * k0 if ctx.needs_input_grad[2] else None
        return dgates, dh0, dc0, None, d_w
