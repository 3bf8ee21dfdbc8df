"""Loss nodes: CTC head (ctc.py:72-97), LabelSmoothingLoss + th_accuracy
(label_smoothing_loss.py:41-63, nets_utils.py:304-324) and the hybrid combination
(espnet_model.py:320-325).  Gradient scales are read from device memory (the autograd
grad_output), so nothing here synchronises with the host."""
from __future__ import annotations

import contextlib

import torch

from .common import F32, empty, lib, ops


def _g(t):
    t = t.contiguous()
    if t.dtype != F32:
        raise RuntimeError("loss gradients must be float32")
    return t


# the CTC head's backward computed in the forward, unscaled, on the auxiliary stream beside the
# latency-bound attention-decoder forward (most CUs idle there); the backward then only scales
# it by the upstream gradient (False: the whole head backward after the decoder's — the path of
# a forward without input gradients; tests/test_trainer_gpu.py compares the two)
CTC_BWD_IN_FWD = True
_ONE = {}


def _one(dev):
    t = _ONE.get(dev)
    if t is None:
        t = _ONE[dev] = torch.ones((), dtype=torch.float32, device=dev)
    return t


class CTCFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, hs, hlens, ys, ylens, ctc, Lmax):
        b = ctc._b
        cd = b.cd
        B, T, d = hs.shape
        V = ctc.ctc_lo.out_features
        dev = hs.device
        N = B * T
        h = empty(N, d, dtype=cd, device=dev)
        logits = empty(N, V, device=dev)
        S = 2 * Lmax + 1
        lse = empty(N, device=dev)
        alpha = torch.empty(B * T * S, dtype=torch.float64, device=dev)
        beta = torch.empty(B * T * S, dtype=torch.float64, device=dev)
        nll = torch.empty(B, dtype=torch.float64, device=dev)
        loss_utt = empty(B, device=dev)
        loss = empty((), device=dev)
        # the whole head (ctc_lo GEMM, log-sum-exp rows, and the lattice: 2 workgroups per
        # utterance for T' serial steps) runs on the auxiliary stream beside the attention
        # decoder's forward (ESPnetASRModel.forward joins before the losses are combined)
        def head():
            ops.scale_dropout(hs.reshape(N, d), h, p=ctc.dropout_rate, seed=ctc._seed)
            ops.linear(h, b.w("ctc_lo.weight"), logits, epi=ops.make_epi(bias=b.f("ctc_lo.bias")))

        pre = CTC_BWD_IN_FWD and ctx.needs_input_grad[0]
        with (ops.aux(hs, h, logits, hlens, ys, ylens, lse, alpha, beta, nll, loss_utt, loss) if ctc._overlap
              else contextlib.nullcontext()):
            head()
            lib.ea_ctc_loss_fwd(B, T, V, logits.data_ptr(), V, hlens.data_ptr(), ys.data_ptr(), ys.stride(0),
                                ylens.data_ptr(), Lmax, lse.data_ptr(), alpha.data_ptr(), beta.data_ptr(),
                                nll.data_ptr(), loss_utt.data_ptr(), loss.data_ptr(), ops.stream())
            if pre:
                # d loss_ctc / d logits for an upstream gradient of 1 (ctc.py:72-97 backward),
                # and through ctc_lo: dh (+ the head's dropout), dW, db — all linear in the
                # upstream gradient, which the backward multiplies in (ea_scale_by_scalar,
                # ea_axpy_dev).  The logits / lattice buffers are released here, not kept.
                dl = empty(N, V, dtype=cd, device=dev)
                lib.ea_ctc_loss_bwd(B, T, V, logits.data_ptr(), V, hlens.data_ptr(), ys.data_ptr(), ys.stride(0),
                                    ylens.data_ptr(), Lmax, lse.data_ptr(), alpha.data_ptr(), beta.data_ptr(),
                                    nll.data_ptr(), _one(dev).data_ptr(), 1.0 / B, dl.data_ptr(), ops.dt(dl), V,
                                    ops.stream())
                dW = empty(V, d, device=dev)
                db = empty(V, device=dev)
                ops.linear_dw(dl, h, dW, accumulate=False)
                ops.colsum(dl, db, accumulate=False, defer=False)
                dh = empty(N, d, device=dev)
                ops.linear_dx(dl, b.w("ctc_lo.weight"), dh)
                if ctc.dropout_rate > 0:
                    ops.scale_dropout(dh, dh, p=ctc.dropout_rate, seed=ctc._seed)
                del dl
        ctx.ctc = ctc
        ctx.meta = (B, T, V, Lmax, d)
        ctx.pre = pre
        if pre:
            main = torch.cuda.current_stream()
            for t in (dh, dW, db):
                t.record_stream(main)  # read by the backward on the main stream
            ctx.save = (dh, dW, db)
        else:
            ctx.save = (h, logits, lse, alpha, beta, nll, hlens, ys, ylens)

        return loss

    @staticmethod
    def backward(ctx, gl):
        ctc = ctx.ctc
        b = ctc._b
        cd = b.cd
        B, T, V, Lmax, d = ctx.meta
        if ctx.pre:  # the head's gradients were computed in the forward for gl = 1: scale them
            dh, dW, db = ctx.save
            ctx.save = None
            gl = _g(gl)
            ops.take_aux_fork()
            st = ops.stream()
            lib.ea_scale_by_scalar(dh.numel(), dh.data_ptr(), gl.data_ptr(), 1.0, st)
            lib.ea_axpy_dev(dW.numel(), dW.data_ptr(), b.g("ctc_lo.weight").data_ptr(), gl.data_ptr(), 1.0, st)
            lib.ea_axpy_dev(V, db.data_ptr(), b.g("ctc_lo.bias").data_ptr(), gl.data_ptr(), 1.0, st)
            ops.grad_ready(b)
            return dh.view(B, T, d), None, None, None, None, None
        h, logits, lse, alpha, beta, nll, hlens, ys, ylens = ctx.save
        ctx.save = None
        N = B * T
        dev = gl.device
        gl = _g(gl)
        # hybrid loss: the autograd engine issues this node after the whole attention decoder
        # backward; forked from the point where the loss gradients exist (CombineFn.backward)
        # onto the auxiliary stream, its kernels fill the CUs the latency-bound decoder
        # backward leaves idle, and the main stream joins before it consumes dh.  dl / dh come
        # from the auxiliary stream's pool: a main-stream block could still be in use by the
        # decoder kernels queued after the fork point.
        fork = ops.take_aux_fork() if ctc._overlap else None
        with (ops.aux(gl, logits, hlens, ys, ylens, lse, alpha, beta, nll, h, after=fork)
              if fork is not None else contextlib.nullcontext()):
            dl = empty(N, V, dtype=cd, device=dev)
            dh = empty(N, d, device=dev)
            lib.ea_ctc_loss_bwd(B, T, V, logits.data_ptr(), V, hlens.data_ptr(), ys.data_ptr(), ys.stride(0),
                                ylens.data_ptr(), Lmax, lse.data_ptr(), alpha.data_ptr(), beta.data_ptr(),
                                nll.data_ptr(), gl.data_ptr(), 1.0 / B, dl.data_ptr(), ops.dt(dl), V,
                                ops.stream())
            with ops.wgrad(dl, h):
                ops.colsum(dl, b.g("ctc_lo.bias"))
                ops.linear_dw(dl, h, b.g("ctc_lo.weight"), accumulate=True)
            ops.linear_dx(dl, b.w("ctc_lo.weight"), dh)
            if ctc.dropout_rate > 0:
                ops.scale_dropout(dh, dh, p=ctc.dropout_rate, seed=ctc._seed)
        if fork is not None:
            ops.join_aux()
            dh.record_stream(torch.cuda.current_stream())  # consumed on the main stream
        ops.grad_ready(b)
        return dh.view(B, T, d), None, None, None, None, None


class LabelSmoothingLossFn(torch.autograd.Function):
    """-> (loss, acc); acc is not differentiable."""

    @staticmethod
    def forward(ctx, x, target, crit):
        B, L, V = x.shape
        rows = B * L
        dev = x.device
        x2 = x.reshape(rows, V)
        lse = empty(rows, device=dev)
        loss_row = torch.empty(rows, dtype=torch.float64, device=dev)
        stat = torch.empty(2, dtype=torch.int32, device=dev)
        loss = empty((), device=dev)
        acc = empty((), device=dev)
        inv = empty(1, device=dev)
        tgt = target.reshape(rows).contiguous()
        lib.ea_lsm_loss_fwd(rows, V, x2.data_ptr(), V, tgt.data_ptr(), crit.smoothing, crit.padding_idx,
                            int(crit.normalize_length), float(B), lse.data_ptr(), loss_row.data_ptr(),
                            stat.data_ptr(), loss.data_ptr(), acc.data_ptr(), inv.data_ptr(), ops.stream())
        ctx.save = (x2, tgt, lse, inv, crit)
        ctx.shape = (B, L, V)
        ctx.mark_non_differentiable(acc)
        return loss, acc

    @staticmethod
    def backward(ctx, gloss, gacc):
        x2, tgt, lse, inv, crit = ctx.save
        ctx.save = None
        B, L, V = ctx.shape
        grad = empty(B, L, V, device=x2.device)
        lib.ea_lsm_loss_bwd(B * L, V, x2.data_ptr(), V, tgt.data_ptr(), crit.smoothing, crit.padding_idx,
                            lse.data_ptr(), _g(gloss).data_ptr(), inv.data_ptr(), 1.0, grad.data_ptr(),
                            0, V, ops.stream())
        return grad, None, None


class CombineFn(torch.autograd.Function):
    """loss = w*a + (1-w)*b  (espnet_model.py:325)."""

    @staticmethod
    def forward(ctx, a, b, w):
        out = empty((), device=a.device)
        lib.ea_axpby_scalar(a.data_ptr(), w, b.data_ptr(), 1.0 - w, out.data_ptr(), ops.stream())
        ctx.w = w
        return out

    @staticmethod
    def backward(ctx, g):
        g = _g(g)
        ga = empty((), device=g.device)
        gb = empty((), device=g.device)
        lib.ea_axpby_scalar(g.data_ptr(), ctx.w, 0, 0.0, ga.data_ptr(), ops.stream())
        lib.ea_axpby_scalar(g.data_ptr(), 1.0 - ctx.w, 0, 0.0, gb.data_ptr(), ops.stream())
        ops.mark_aux_fork()  # the CTC head's backward forks from here (CTCFn.backward)
        return ga, gb, None
