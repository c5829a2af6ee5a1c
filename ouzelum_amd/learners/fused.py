"""GPU-side building blocks of the recurrent learner (HIP + hipBLASLt), with autograd.

* ``LSTMSequence``: the whole done-masked recurrence of ``RPO-LSTM/model.py:34-50`` over T
  steps.  For the reference's hidden size 128: ONE launch forward (``ouz_lstm_seq_fwd``) and one for BPTT
  (``ouz_lstm_seq_bwd``), each workgroup carrying 16 batch rows through all T steps with the recurrent product
  on the f32 MFMA (round 6).  Otherwise per step one hipBLASLt GEMM (h W_hh^T added onto the precomputed input
  projection) and ONE fused HIP cell kernel (``ouz_lstm_cell_fwd``); BPTT is the mirror image
  (``ouz_lstm_cell_bwd`` + one GEMM per step).  dW_hh is one split-K product over all T·B rows either way.
  torch's per-step nn.LSTM costs ~10 element-wise launches forward and ~20 backward per step.
* ``splitk_wgrad`` / ``SplitKLinear``: weight gradients dW = dYᵀ X with K = T·B rows
  (32 768 at the reference's 16 x 4096 minibatch halves) and a small output (512 x 256):
  a plain GEMM puts 16 output tiles on 256 CUs; splitting K into S slabs and summing
  gives 16·S workgroups.
* ``LinearTanh``: Linear + Tanh of the MLP trunks with the backward's tanh' and bias
  gradient in one HIP pass (``ouz_tanh_bwd_bias``) instead of tanh_backward + a column sum.
* ``PolicyLoss`` / ``ValueLoss``: the PPO losses of a minibatch (``RPO-LSTM/agent.py:86-110``)
  as one HIP forward each that also writes the loss's input gradients (``ouz_ppo_policy_loss``,
  ``ouz_ppo_value_loss``), replacing ~60 element-wise and reduction launches per minibatch.
"""
import os

import torch

from .. import _lib as L

_INPLACE_GATES = os.environ.get("OUZ_LSTM_INPLACE_GATES", "1") != "0"
# the whole recurrence in one launch each way (ouz_lstm_seq_fwd / _bwd) where H = 128; OUZ_LSTM_SEQ=0 keeps the
# per-step GEMM + cell kernel pairs
_SEQ = os.environ.get("OUZ_LSTM_SEQ", "1") != "0"
SEQ_H = 128
_FUSED_TANH = os.environ.get("OUZ_FUSED_TANH", "1") != "0"
_FUSED_SAMPLE = os.environ.get("OUZ_FUSED_SAMPLE", "1") != "0"
# the trunks' first layer (K <= 16 inputs) + tanh in one HIP pass (ouz_linear_tanh_small_k); OUZ_SMALLK_TANH=0 keeps
# hipBLASLt's GEMM + torch's tanh
_SMALLK_TANH = os.environ.get("OUZ_SMALLK_TANH", "1") != "0"


_SPLITK = os.environ.get("OUZ_SPLITK", "1") != "0"


def _splits(k, n_out_tiles):
    """Number of K slabs: enough workgroups to cover the chip, slabs of >= 256 rows (OUZ_SPLITK=0: one plain GEMM)."""
    if not _SPLITK:
        return 1
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


def smallk_ok(x, weight, bias):
    """``linear_tanh_small_k`` applies: f32 CUDA rows, K <= 16 inputs, a power-of-two width in [4, 1024], a bias."""
    cols, k = weight.shape
    return (_SMALLK_TANH and bias is not None and x.is_cuda and x.dtype == torch.float32 and x.dim() == 2
            and 1 <= k <= 16 and 4 <= cols <= 1024 and cols & (cols - 1) == 0)


def linear_tanh_small_k(x, weight, bias):
    """tanh(x Wᵀ + b) for a first layer of K <= 16 inputs in one pass (``ouz_linear_tanh_small_k``; no autograd)."""
    x = x.contiguous()
    w, b = weight.detach().contiguous(), bias.detach().contiguous()
    y = torch.empty((x.shape[0], w.shape[0]), device=x.device)
    L.check(L.lib.ouz_linear_tanh_small_k(x.data_ptr(), w.data_ptr(), b.data_ptr(), x.shape[0], w.shape[1], w.shape[0],
                                          y.data_ptr(), L.stream_ptr(x.device)), "ouz_linear_tanh_small_k")
    return y


class LinearTanh(torch.autograd.Function):
    """y = tanh(x Wᵀ + b) (one HIP pass where K <= 16: ``linear_tanh_small_k``); backward: dz = dy (1 - y²) and
    db = Σ_rows dz in one HIP pass, then dx = dz W and the split-K dW = dzᵀ x."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        if smallk_ok(x, weight, bias):
            y = linear_tanh_small_k(x, weight, bias)
        else:
            y = torch.addmm(bias, x, weight.t())
            torch.tanh_(y)
        ctx.save_for_backward(x, weight, y)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight, y = ctx.saved_tensors
        dy = dy.contiguous()
        rows, cols = y.shape
        dz = torch.empty_like(y)
        db = torch.empty(cols, device=y.device)
        ws = torch.empty(L.COLSUM_BLOCKS * cols, device=y.device)
        L.check(L.lib.ouz_tanh_bwd_bias(dy.data_ptr(), y.data_ptr(), rows, cols, ws.data_ptr(), dz.data_ptr(),
                                        db.data_ptr(), L.stream_ptr(y.device)), "ouz_tanh_bwd_bias")
        dx = dz.mm(weight) if ctx.needs_input_grad[0] else None
        dw = splitk_wgrad(dz, x.contiguous()) if ctx.needs_input_grad[1] else None
        return dx, dw, db


def _fused_ok(x, min_rows):
    return x.is_cuda and x.dim() == 2 and x.shape[0] >= min_rows and torch.is_grad_enabled()


def linear(x, layer, min_rows=8192):
    """nn.Linear forward; rows >= min_rows on a GPU take the split-K weight gradient."""
    if _fused_ok(x, min_rows):
        return SplitKLinear.apply(x, layer.weight, layer.bias)
    return torch.nn.functional.linear(x, layer.weight, layer.bias)


def _tanh_fusable(layer, x, min_rows):
    cols = layer.out_features
    return (_FUSED_TANH and layer.bias is not None and _fused_ok(x, min_rows) and 4 <= cols <= 1024
            and cols & (cols - 1) == 0)


def run_mlp(seq, x, min_rows=8192):
    """Forward through an nn.Sequential of Linear / activation modules using ``linear``; a Linear followed by a
    Tanh becomes one ``LinearTanh`` where its rows and width allow, and, without autograd (the rollout's policy and
    value calls), a first layer of K <= 16 inputs + its Tanh one ``linear_tanh_small_k`` pass at any row count."""
    mods = list(seq)
    i = 0
    while i < len(mods):
        m = mods[i]
        if isinstance(m, torch.nn.Linear) and i + 1 < len(mods) and isinstance(mods[i + 1], torch.nn.Tanh):
            if _tanh_fusable(m, x, min_rows):
                x = LinearTanh.apply(x, m.weight, m.bias)
                i += 2
                continue
            if not torch.is_grad_enabled() and smallk_ok(x, m.weight, m.bias):
                x = linear_tanh_small_k(x, m.weight, m.bias)
                i += 2
                continue
        x = linear(x, m, min_rows) if isinstance(m, torch.nn.Linear) else m(x)
        i += 1
    return x


class PolicyLoss(torch.autograd.Function):
    """(mean_z (n, 4), logstd (1, 4), actions (n, 4), old_logp (n,), advantages (n,), clip, norm_adv) ->
    (pg_loss, approx_kl, clipfrac), 0-dim; only pg_loss is differentiable.  ``mean_z`` is the policy mean with
    RPO's noise already added (model.py:61-64)."""

    @staticmethod
    def forward(ctx, mean_z, logstd, actions, old_logp, adv, clip, norm_adv):
        dev = mean_z.device
        n = mean_z.shape[0]
        # contiguous f32 operands held in locals until the launch is queued
        mz, ls, act, old, a = (t.detach().contiguous() for t in (mean_z, logstd, actions, old_logp, adv))
        for t, name in ((mz, "mean_z"), (ls, "logstd"), (act, "actions"), (old, "old_logp"), (a, "advantages")):
            L.require_hip_tensor(t, name)
            if t.dtype != torch.float32:
                raise ValueError(f"PolicyLoss: {name} must be float32")
        if mz.shape != (n, L.NUM_ACT) or act.shape != (n, L.NUM_ACT) or ls.numel() != L.NUM_ACT \
                or old.numel() != n or a.numel() != n:
            raise ValueError("PolicyLoss: mean_z / actions (n, 4), logstd 4 values, old_logp / advantages n values")
        dmean = torch.empty_like(mz)
        loss, kl, cf = (torch.empty((), device=dev) for _ in range(3))
        dls = torch.empty(logstd.shape, device=dev)
        ws = torch.empty(L.LOSS_WS_DOUBLES, dtype=torch.float64, device=dev)
        L.check(L.lib.ouz_ppo_policy_loss(mz.data_ptr(), ls.data_ptr(), act.data_ptr(), old.data_ptr(), a.data_ptr(),
                                          n, float(clip), int(bool(norm_adv)), ws.data_ptr(), dmean.data_ptr(),
                                          loss.data_ptr(), kl.data_ptr(), cf.data_ptr(), dls.data_ptr(),
                                          L.stream_ptr(dev)), "ouz_ppo_policy_loss")
        ctx.save_for_backward(dmean, dls)
        ctx.mark_non_differentiable(kl, cf)
        ctx.set_materialize_grads(False)
        return loss, kl, cf

    @staticmethod
    def backward(ctx, g, _gkl, _gcf):
        dmean, dls = ctx.saved_tensors
        return dmean * g, dls * g, None, None, None, None, None


class ValueLoss(torch.autograd.Function):
    """(values (n,), returns (n,)) -> 0.5 * mean((values - returns)²), 0-dim (agent.py:104-105)."""

    @staticmethod
    def forward(ctx, values, returns):
        dev = values.device
        v, r = values.detach().contiguous(), returns.detach().contiguous()
        L.require_hip_tensor(v, "values")
        L.require_hip_tensor(r, "returns")
        if v.dim() != 1 or r.shape != v.shape or v.dtype != torch.float32 or r.dtype != torch.float32:
            raise ValueError("ValueLoss: values and returns (n,) float32")
        dv = torch.empty_like(v)
        loss = torch.empty((), device=dev)
        ws = torch.empty(L.LOSS_WS_DOUBLES, dtype=torch.float64, device=dev)
        L.check(L.lib.ouz_ppo_value_loss(v.data_ptr(), r.data_ptr(), v.shape[0], ws.data_ptr(), dv.data_ptr(),
                                         loss.data_ptr(), L.stream_ptr(dev)), "ouz_ppo_value_loss")
        ctx.save_for_backward(dv)
        return loss

    @staticmethod
    def backward(ctx, g):
        (dv,) = ctx.saved_tensors
        return dv * g, None


def policy_sample_ok(hidden, head):
    return (_FUSED_SAMPLE and hidden.is_cuda and not torch.is_grad_enabled() and hidden.dim() == 2
            and hidden.dtype == torch.float32 and hidden.shape[1] % 4 == 0 and head.out_features == L.NUM_ACT
            and head.bias is not None)


def policy_sample(hidden, head, logstd, eps):
    """The rollout policy's mean head + sample in one HIP launch (``ouz_policy_sample``): (action, log-prob,
    entropy) as ``models._sample_head(head(hidden), logstd, eps)``."""
    B, H = hidden.shape
    dev = hidden.device
    h = hidden.contiguous()
    w, b, ls, e = (t.detach().contiguous() for t in (head.weight, head.bias, logstd, eps))
    action = torch.empty((B, L.NUM_ACT), device=dev)
    logprob = torch.empty(B, device=dev)
    entropy = torch.empty(B, device=dev)
    L.check(L.lib.ouz_policy_sample(h.data_ptr(), w.data_ptr(), b.data_ptr(), ls.data_ptr(), e.data_ptr(), B, H,
                                    action.data_ptr(), logprob.data_ptr(), entropy.data_ptr(), L.stream_ptr(dev)),
            "ouz_policy_sample")
    return action, logprob, entropy


def _p(t):
    return None if t is None else t.data_ptr()


SEQ_MIN_T = 4


def seq_kernels_ok(x_proj, *bufs):
    """The fused sequence kernels apply: hidden size 128 (the reference actor's), f32, and a sequence of at least
    SEQ_MIN_T steps.  Each workgroup loads its 256 KB of weight fragments once per launch and keeps them in registers,
    which pays over a sequence (the update's T = 16); the rollout's one-step policy calls keep the GEMM + cell pair.
    ``bufs``: caller-owned output buffers (the in-place carry), which the kernels need 16-byte aligned."""
    return (_SEQ and x_proj.shape[-1] == 4 * SEQ_H and x_proj.dtype == torch.float32
            and x_proj.shape[0] >= SEQ_MIN_T and all(b.data_ptr() % 16 == 0 for b in bufs))


def _a16(t):
    """t, or an aligned copy: the sequence kernels make one 16-byte access per lane (a tensor that is a view at an
    odd offset into a larger buffer is copied)."""
    return t if t is None or t.data_ptr() % 16 == 0 else t.clone()


def seq_pack(w_hh):
    """W_hh in the sequence kernels' two fragment layouts (ouz_lstm_seq_pack): (w_fwd, w_bwd)."""
    w = w_hh.detach().contiguous()
    wf, wb = torch.empty_like(w), torch.empty_like(w)
    L.check(L.lib.ouz_lstm_seq_pack(w.data_ptr(), w.shape[1], wf.data_ptr(), wb.data_ptr(), L.stream_ptr(w.device)),
            "ouz_lstm_seq_pack")
    return wf, wb


def _lstm_forward_seq(x_proj, h0, c0, keep, w_hh, carry_out=None, saved=True, packed=None):
    """``_lstm_forward`` as ONE launch (ouz_lstm_seq_fwd): the carry stays on chip across the T steps.  ``saved=False``
    (inference) skips the tensors only BPTT reads.  ``packed``: seq_pack(w_hh), made here when not given."""
    T, B, G4 = x_proj.shape
    H = G4 // 4
    dev = x_proj.device
    x_proj = _a16(x_proj.contiguous())
    keep = keep.contiguous().float()
    h0, c0 = h0.contiguous(), _a16(c0.contiguous())
    w = (packed or seq_pack(w_hh))[0]
    hid = torch.empty((T, B, H), device=dev)
    act = c_all = hm = cm = None
    if saved:
        act = torch.empty((T, B, G4), device=dev)
        c_all = torch.empty((T, B, H), device=dev)
        hm = torch.empty((T + 1, B, H), device=dev)
        cm = torch.empty((T + 1, B, H), device=dev)
    ho, co = carry_out if carry_out is not None else (None, None)
    L.check(L.lib.ouz_lstm_seq_fwd(x_proj.data_ptr(), h0.data_ptr(), c0.data_ptr(), keep.data_ptr(), w.data_ptr(),
                                   T, B, H, _p(act), _p(c_all), hid.data_ptr(), _p(hm), _p(cm), _p(ho), _p(co),
                                   L.stream_ptr(dev)), "ouz_lstm_seq_fwd")
    return act, c_all, hid, hm, cm, keep


def _lstm_forward(x_proj, h0, c0, keep, w_hh, carry_out=None, saved=True):
    """The T-step recurrence: per step the recurrent GEMM onto the input projection and one fused cell launch
    (or all T steps in one launch, ``_lstm_forward_seq``, where ``seq_kernels_ok``).  Returns (act, c_all, hid, hm,
    cm, keep).  ``carry_out=(h, c)``: the last step writes the final carry (keep = 1, so the masked next-step carry is
    the carry itself) into these buffers instead of the scratch row; they may alias h0 / c0, which are consumed
    (masked into hm[0] / cm[0]) before any cell launch."""
    if seq_kernels_ok(x_proj, *(carry_out or ())):
        return _lstm_forward_seq(x_proj, h0, c0, keep, w_hh, carry_out, saved)
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
            # copy launch per step.  x_proj is the caller's own temporary (SplitKLinear / addmm output)
            # and is not saved for the backward pass.
            gates = x_proj[t]
            torch.addmm(gates, hm[t], w_t, out=gates)
        else:
            torch.addmm(x_proj[t], hm[t], w_t, out=gates)
        kn = keep[t + 1] if t + 1 < T else None
        h_next, c_next = hm[t + 1], cm[t + 1]
        if carry_out is not None and t == T - 1:
            h_next, c_next = carry_out
        L.check(L.lib.ouz_lstm_cell_fwd(gates.data_ptr(), cm[t].data_ptr(), _p(kn), act[t].data_ptr(),
                                        c_all[t].data_ptr(), hid[t].data_ptr(), h_next.data_ptr(),
                                        c_next.data_ptr(), B, H, stream), "ouz_lstm_cell_fwd")
    return act, c_all, hid, hm, cm, keep


def lstm_sequence_carry_inplace(x_proj, h0, c0, keep, w_hh, h_out, c_out):
    """Inference form of ``LSTMSequence`` (no autograd): returns hid (T, B, H) and writes the final carry into
    h_out / c_out (contiguous (B, H) buffers, which may be h0 / c0 themselves) instead of returning copies.  The
    graphed rollout policy keeps its carry in its static input buffers this way: no copy in or out per step."""
    for t, name in ((h_out, "h_out"), (c_out, "c_out")):
        if not t.is_contiguous() or tuple(t.shape[-2:]) != (x_proj.shape[1], x_proj.shape[2] // 4):
            raise ValueError(f"lstm_sequence_carry_inplace: {name} must be a contiguous (B, H) buffer")
    return _lstm_forward(x_proj, h0, c0, keep, w_hh, carry_out=(h_out, c_out), saved=False)[2]


class LSTMSequence(torch.autograd.Function):
    """(x_proj (T,B,4H), h0 (B,H), c0 (B,H), keep (T,B), W_hh (4H,H)) -> (hidden (T,B,H), h_T, c_T).
    keep[t] = 1 - done[t] zeroes the carry entering step t (model.py:42-46)."""

    @staticmethod
    def forward(ctx, x_proj, h0, c0, keep, w_hh):
        ctx.set_materialize_grads(False)     # unused h_T / c_T come back as None, not zero-filled tensors
        packed = seq_pack(w_hh) if seq_kernels_ok(x_proj) else None
        act, c_all, hid, hm, cm, keep = (_lstm_forward_seq(x_proj, h0, c0, keep, w_hh, packed=packed) if packed
                                         else _lstm_forward(x_proj, h0, c0, keep, w_hh))
        ctx.packed_bwd = packed[1] if packed else None
        ctx.save_for_backward(act, c_all, cm, hm, keep, w_hh)
        T = hid.shape[0]
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
        if ctx.packed_bwd is not None:
            # BPTT of all T steps in one launch (ouz_lstm_seq_bwd); dW_hh stays one split-K product over T·B rows
            wt = ctx.packed_bwd
            ctx.packed_bwd = None
            dh0 = torch.empty((B, H), device=dev) if ctx.needs_input_grad[1] else None
            dc0 = torch.empty((B, H), device=dev) if ctx.needs_input_grad[2] else None
            dhid, dhT, dcT = _a16(dhid), _a16(dhT), _a16(dcT)
            L.check(L.lib.ouz_lstm_seq_bwd(act.data_ptr(), c_all.data_ptr(), cm.data_ptr(), keep.data_ptr(),
                                           wt.data_ptr(), dhid.data_ptr(), _p(dhT), _p(dcT), T, B, H,
                                           dgates.data_ptr(), _p(dh0), _p(dc0), stream), "ouz_lstm_seq_bwd")
            d_w = (splitk_wgrad(dgates.view(T * B, G4), hm[:T].reshape(T * B, H)) if ctx.needs_input_grad[4]
                   else None)
            return dgates, dh0, dc0, None, d_w
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


class ClipAdam:
    """``nn.utils.clip_grad_norm_(params, max_norm)`` + ``optimizer.step()`` (RPO-LSTM/agent.py:124-134) as two HIP
    launches (``ouz_adam_clip_step``) instead of torch's per-tensor norms, their stack / norm / clamp / scale and the
    multi-tensor Adam kernel.  ``optimizer`` is a plain ``torch.optim.Adam`` (one parameter group, f32 CUDA
    parameters, no weight decay / amsgrad / maximize): it keeps the parameter group, the hyper-parameters and the
    state (``step`` on the host, ``exp_avg``, ``exp_avg_sq``), so its ``state_dict`` / ``load_state_dict`` are the
    reference's checkpoint files unchanged; only its ``step`` is replaced.  The clipped gradients are not written
    back into ``.grad`` (nothing reads them after the step)."""

    def __init__(self, optimizer):
        (group,) = optimizer.param_groups
        if (group["weight_decay"] or group["amsgrad"] or group["maximize"] or len(group["params"]) > L.ADAM_MAX_TENSORS
                or any(p.dtype != torch.float32 or p.device.type != "cuda" for p in group["params"])):
            raise ValueError("ClipAdam: one group of <= 16 f32 CUDA tensors, plain Adam")
        self.optimizer = optimizer
        self.device = group["params"][0].device
        self.ws = torch.empty(L.ADAM_WS_FLOATS, device=self.device)

    def step(self, max_norm):
        (group,) = self.optimizer.param_groups
        table = L.OuzAdamTable()
        keep = []
        n, step = 0, None
        for p in group["params"]:
            if p.grad is None:
                continue
            st = self.optimizer.state[p]
            if not st:   # torch's lazy state (Adam._init_group, non-fused form: the step count on the host)
                st["step"] = torch.tensor(0.0, dtype=torch.float32)
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            if st["step"].device.type != "cpu":
                st["step"] = st["step"].cpu()
            st["step"] += 1
            s = int(st["step"])
            if step is None:
                step = s
            elif s != step:
                raise ValueError("ClipAdam: parameters at different Adam step counts")
            g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
            keep.append(g)
            table.numel[n] = p.numel()
            table.grad[n], table.param[n] = g.data_ptr(), p.data_ptr()
            table.exp_avg[n], table.exp_avg_sq[n] = st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr()
            n += 1
        if n == 0:
            return
        table.n_tensors = n
        b1, b2 = group["betas"]
        L.check(L.lib.ouz_adam_clip_step(table, float(group["lr"]), float(b1), float(b2), float(group["eps"]), step,
                                         float(max_norm or 0.0), self.ws.data_ptr(), L.stream_ptr(self.device)),
                "ouz_adam_clip_step")


_FOREACH_COPY = os.environ.get("OUZ_FOREACH_COPY", "1") != "0"


def store(dsts, srcs):
    """dst.copy_(src) for each pair, as ONE multi-tensor launch (torch._foreach_copy_) where all are CUDA tensors of
    one dtype: the rollout loop's per-step storage writes (5 copies per step: 20 against 8.6 µs,
    ``scripts/exp/copy_gather_probe.py``); ``OUZ_FOREACH_COPY=0`` keeps one copy each."""
    if (_FOREACH_COPY and all(t.is_cuda for t in (*dsts, *srcs))
            and len({t.dtype for t in (*dsts, *srcs)}) == 1):
        torch._foreach_copy_(list(dsts), list(srcs))
    else:
        for d, s in zip(dsts, srcs):
            d.copy_(s)
