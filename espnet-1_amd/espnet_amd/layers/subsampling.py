"""Conv2dSubsampling (espnet/nets/pytorch_backend/transformer/subsampling.py:46-91) +
RelPositionalEncoding (transformer/embedding.py:260-331), MI355X layout.

The reference runs NCHW Conv2d(1,d,3,2)+ReLU, Conv2d(d,d,3,2)+ReLU, then
x.transpose(1,2).view(b, t, c*f) -> Linear(d*F'', d) -> x*sqrt(d) -> dropout.
Here activations are channel-last (B, T, F, C): both convolutions are MFMA GEMMs over
im2col rows (conv1: 9 taps padded to 16; conv2: K = 9*C, the implicit-GEMM hot spot that
is ~32% of the step's FLOPs), ReLU fused in the GEMM epilogue, and the Linear consumes
the (t, f*C + c) order directly — its weight (d, C, F'') is repacked to (d, F'', C) per step
(5 M elements) instead of transposing the 310 MB activation.
"""
from __future__ import annotations

import ctypes
import math
import os

import torch
from torch import nn

from .._lib import CONV_DGRAD, CONV_FWD, CONV_WGRAD, GEMM_PIPE, ConvGeo
from .common import (ACT_RELU, EPI_ACT, EPI_DACT, EPI_STORE, F32, Bound, empty, lib, ops, rup)


def phase_geo(B, T1, F1, T2, F2, C, mode, a=0, e=0, zero=0):
    """ea_conv_geo of the phase-split conv1 output x1p (include/espnet_amd.h): class plane
    (a, e) holds pixels t1 = 2i+a, f1 = 2j+e as [b][i][j][C]."""
    g = ConvGeo()
    g.mode, g.B, g.T2, g.F2, g.C, g.P = mode, B, T2, F2, C, B * T2 * F2
    nI = ((T1 + 1) // 2, T1 // 2)
    nJ = ((F1 + 1) // 2, F1 // 2)
    g.nI[0], g.nI[1] = nI
    g.nJ[0], g.nJ[1] = nJ
    rows = [B * nI[0] * nJ[0], B * nI[0] * nJ[1], B * nI[1] * nJ[0], B * nI[1] * nJ[1]]
    off = 0
    for i in range(4):
        g.plane[i] = off * C
        off += rows[i]
    g.a, g.e, g.zero = a, e, zero
    return g, nI, nJ, rows


# conv1's weight gradient fused into conv2's input-gradient epilogue (ea_gemm_conv_w1)
FUSE_CONV1_WGRAD = os.environ.get("EA_FUSE_CONV1_WGRAD", "1") != "0"
# ... with conv1's ReLU mask from support bits written by the forward (else the bf16 x1p rows)
CONV1_POS_BITS = os.environ.get("EA_CONV1_POS_BITS", "1") != "0"
# ... and the four parity classes in one launch (False: one launch per class, the path with
# EA_GEMM_PIPE=0 since the merged launch is a gemm_pipe kernel; tests compare the two)
MERGED_DGRAD = GEMM_PIPE != 0
# ... reading conv2's weight K-major, W2k [ci][tap][co] (False: W2t [tap][co][ci], bit-identical)
DGRAD_KMAJOR = True


def _implicit_ok(cd, C):
    return cd == torch.bfloat16 and C % 64 == 0 and 256 % (C // 8) == 0


def rel_pos_table(n, d):
    """RelPositionalEncoding.extend_pe (embedding.py:282-313): rows = relative positions
    n-1 ... -(n-1).  A constant computed once at construction, like the reference."""
    pos = torch.arange(0, n, dtype=torch.float32).unsqueeze(1)
    div = torch.exp(torch.arange(0, d, 2, dtype=torch.float32) * -(math.log(10000.0) / d))
    pp = torch.zeros(n, d)
    pn = torch.zeros(n, d)
    pp[:, 0::2] = torch.sin(pos * div)
    pp[:, 1::2] = torch.cos(pos * div)
    pn[:, 0::2] = torch.sin(-1 * pos * div)
    pn[:, 1::2] = torch.cos(-1 * pos * div)
    return torch.cat([torch.flip(pp, [0]), pn[1:]], 0)


class RelPositionalEncoding(nn.Module):
    """Holds the constant table; forward returns dropout(table slice) in the compute dtype."""

    def __init__(self, d_model, dropout_rate, max_len=5000):
        super().__init__()
        self.d_model = d_model
        self.xscale = math.sqrt(d_model)
        self.dropout_rate = dropout_rate
        self.max_len = max_len
        self._pe = None  # device copy, built lazily (not a buffer: not in the state_dict)

    def table(self, T, device):
        n = max(self.max_len, T)
        if self._pe is None or self._pe.shape[0] < 2 * T - 1 or self._pe.device != device:
            self._pe = rel_pos_table(n, self.d_model).to(device)
        return self._pe

    def pos_emb(self, T, device, cd, training, seed):
        pe = self.table(T, device)
        c = pe.shape[0] // 2
        src = pe[c - T + 1: c + T]
        out = empty(2 * T - 1, self.d_model, dtype=cd, device=device)
        ops.scale_dropout(src, out, 1.0, self.dropout_rate if training else 0.0, seed)
        return out


class Conv2dSubsampling(nn.Module):
    """Parameter holder with the reference's names: conv.0 / conv.2 / out.0 (+ pos_enc)."""

    def __init__(self, idim, odim, dropout_rate, pos_enc=None):
        super().__init__()
        self.conv = nn.Sequential(nn.Conv2d(1, odim, 3, 2), nn.ReLU(), nn.Conv2d(odim, odim, 3, 2), nn.ReLU())
        self.F1 = (idim - 1) // 2
        self.F2 = (self.F1 - 1) // 2
        self.out = nn.Sequential(nn.Linear(odim * self.F2, odim),
                                 pos_enc if pos_enc is not None else RelPositionalEncoding(odim, dropout_rate))
        self.odim = odim
        self.idim = idim
        self._b = None

    def bind(self, arena, prefix, cd):
        self._b = Bound(arena, prefix, cd)

    def forward(self, feats, seed):
        return SubsampleFn.apply(feats, self._anchor, self, seed, self.training)


def _out_linear(x2r, wl, b, pe, p, seed, B, T2, C):
    """out.0 Linear on (t, f*C + c) rows, then x*sqrt(d) and dropout (embedding.py:326 for
    RelPositionalEncoding); with the absolute PositionalEncoding (TransformerEncoder) the
    table row is added before the dropout (embedding.py:91-92).  Both apply the dropout
    with ea_scale_dropout's index law, so the backward is the same scale-dropout."""
    y = empty(B * T2, C, device=x2r.device)
    if getattr(pe, "absolute", False):
        ops.linear(x2r, wl, y, epi=ops.make_epi(bias=b.f("out.0.bias"), post_scale=pe.xscale))
        lib.ea_add_pe_dropout(B * T2, C, T2, pe.table(T2, y.device).data_ptr(), float(p), seed, y.data_ptr(),
                              ops.stream())
    else:
        ops.linear(x2r, wl, y, epi=ops.make_epi(bias=b.f("out.0.bias"), post_scale=pe.xscale, drop_p=p, seed=seed))
    return y


class SubsampleFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, feats, anchor, m: Conv2dSubsampling, seed, training):
        b = m._b
        cd = b.cd
        B, T, Fin = feats.shape
        C = m.odim
        T1, F1 = (T - 3) // 2 + 1, (Fin - 3) // 2 + 1
        T2, F2 = (T1 - 3) // 2 + 1, (F1 - 3) // 2 + 1
        dev = feats.device
        pe = m.out[1]
        if _implicit_ok(cd, C):
            return SubsampleFn._forward_implicit(ctx, feats, m, seed, training, B, T, Fin, C, T1, F1, T2, F2)
        ctx.implicit = False
        # conv1: im2col (P1 x 16) . W1p^T -> relu -> x1 (B,T1,F1,C)
        P1 = B * T1 * F1
        col1 = empty(P1, 16, dtype=cd, device=dev)
        lib.ea_im2col_conv1(B, T, Fin, feats.data_ptr(), col1.data_ptr(), ops.dt(col1), ops.stream())
        w1 = empty(C, 16, dtype=cd, device=dev)
        w1.zero_()
        ops.scale_dropout(b.f("conv.0.weight", shape=(C, 9)), w1[:, :9])
        x1 = empty(P1, C, dtype=cd, device=dev)
        ops.linear(col1, w1, x1, epi=ops.make_epi(EPI_ACT, bias=b.f("conv.0.bias"), act=ACT_RELU))
        # conv2: im2col (P2 x 9C) . W2p^T -> relu -> x2 (B,T2,F2,C)
        P2 = B * T2 * F2
        col2 = empty(P2, 9 * C, dtype=cd, device=dev)
        lib.ea_im2col_conv2(B, T1, F1, C, x1.data_ptr(), col2.data_ptr(), ops.dt(col2), ops.stream())
        w2 = empty(C, 9 * C, dtype=cd, device=dev)
        ops.permute3(b.f("conv.2.weight"), w2, C, C, 9)  # (Co,Ci,9) -> (Co,9,Ci)
        x2 = empty(P2, C, dtype=cd, device=dev)
        probe = ops.PROBE
        if probe is not None:
            probe.begin("conv2_gemm")
        ops.linear(col2, w2, x2, epi=ops.make_epi(EPI_ACT, bias=b.f("conv.2.bias"), act=ACT_RELU))
        if probe is not None:
            probe.end("conv2_gemm")
        # out.0 Linear on (t, f*C + c) rows, * sqrt(d), dropout (embedding.py:326)
        wl = empty(C, F2 * C, dtype=cd, device=dev)
        ops.permute3(b.f("out.0.weight"), wl, C, C, F2)  # (d, C, F2) -> (d, F2, C)
        p = pe.dropout_rate if training else 0.0
        y = _out_linear(x2.view(B * T2, F2 * C), wl, b, pe, p, seed, B, T2, C)
        ctx.m = m
        ctx.meta = (B, T, Fin, T1, F1, T2, F2, p, seed)
        ctx.save = (col1, x1, col2, w2, x2, wl)
        return y.view(B, T2, C)

    @staticmethod
    def _forward_implicit(ctx, feats, m, seed, training, B, T, Fin, C, T1, F1, T2, F2):
        """bf16 path: conv1 direct into the phase-split x1p, conv2 as an implicit GEMM
        gathering x1p rows (ea_gemm_conv EA_CONV_FWD) — no im2col buffers."""
        b = m._b
        cd = b.cd
        dev = feats.device
        pe = m.out[1]
        P1, P2 = B * T1 * F1, B * T2 * F2
        x1p = empty(P1 + 64, C, dtype=cd, device=dev)  # + 64 zero rows (wgrad gather padding)
        x1p[P1:].zero_()
        # ReLU support bits of x1p for the fused backward's mask (1/16 of x1p's bytes)
        pos1 = (torch.empty(P1 * C // 8, dtype=torch.uint8, device=dev)
                if training and FUSE_CONV1_WGRAD and CONV1_POS_BITS else None)
        lib.ea_conv1_fwd2(B, T, Fin, C, feats.data_ptr(), b.f("conv.0.weight").data_ptr(),
                          b.f("conv.0.bias").data_ptr(), x1p.data_ptr(), ops.dt(x1p),
                          0 if pos1 is None else pos1.data_ptr(), ops.stream())
        # K order (64-channel block, tap, channel): (Co, Ci/64, 64, 9) -> (Co, Ci/64, 9, 64)
        w2 = empty(C, 9 * C, dtype=cd, device=dev)
        ops.permute3(b.f("conv.2.weight"), w2, C * C // 64, 64, 9)
        x2 = empty(P2, C, dtype=cd, device=dev)
        geo, _, _, _ = phase_geo(B, T1, F1, T2, F2, C, CONV_FWD)
        probe = ops.PROBE
        if probe is not None:
            probe.begin("conv2_gemm")
        epi = ops.make_epi(EPI_ACT, bias=b.f("conv.2.bias"), act=ACT_RELU)
        ws = ops.workspace(ops._SPLITK_WS, dev)
        lib.ea_gemm_conv(ctypes.byref(geo), 1, 1, P2, C, 9 * C, x1p.data_ptr(), C, w2.data_ptr(), 9 * C,
                         x2.data_ptr(), ops.dt(x2), C, ctypes.byref(epi), ws.data_ptr(), ws.numel(), ops.stream())
        if probe is not None:
            probe.end("conv2_gemm")
        wl = empty(C, F2 * C, dtype=cd, device=dev)
        ops.permute3(b.f("out.0.weight"), wl, C, C, F2)  # (d, C, F2) -> (d, F2, C)
        p = pe.dropout_rate if training else 0.0
        y = _out_linear(x2.view(B * T2, F2 * C), wl, b, pe, p, seed, B, T2, C)
        ctx.m = m
        ctx.implicit = True
        ctx.meta = (B, T, Fin, T1, F1, T2, F2, p, seed)
        ctx.save = (feats, x1p, w2, x2, wl, pos1)
        return y.view(B, T2, C)

    @staticmethod
    def _backward_implicit(ctx, dy):
        m = ctx.m
        b = m._b
        cd = b.cd
        B, T, Fin, T1, F1, T2, F2, p, seed = ctx.meta
        feats, x1p, w2, x2, wl, pos1 = ctx.save
        ctx.save = None
        C = m.odim
        dev = dy.device
        P1, P2 = B * T1 * F1, B * T2 * F2
        dv = empty(B * T2, C, dtype=cd, device=dev)
        ops.scale_dropout_colsum(dy.reshape(B * T2, C).contiguous(), dv, b.g("out.0.bias"), scale=m.out[1].xscale,
                                 p=p, seed=seed)
        x2r = x2.view(B * T2, F2 * C)
        with ops.wgrad(dv, x2):
            dwl = empty(C, F2 * C, device=dev)
            gw = b.g("out.0.weight")
            ops.linear_dw(dv, x2r, dwl, accumulate=False,  # then (d,F2,C) -> (d,C,F2) into the arena
                          post=lambda: ops.permute3(dwl, gw, C, F2, C, accumulate=True))
        # dY2 (relu-masked) with >= 64 zero rows after P2: the wgrad K padding and the dgrad
        # gather's off-grid rows
        K2 = rup(P2, 64)
        dx2 = empty(P2 + 128, C, dtype=cd, device=dev)
        dx2[P2:].zero_()
        ops.linear_dx(dv, wl, dx2[:P2].view(B * T2, F2 * C), epi=ops.make_epi(EPI_DACT, act=ACT_RELU, aux=x2r))
        ws_side = None
        with ops.wgrad(dx2, x1p, launches=True):
            ops.colsum(dx2[:P2], b.g("conv.2.bias"))
            dw2 = empty(C, 9 * C, device=dev)
            geo, _, _, _ = phase_geo(B, T1, F1, T2, F2, C, CONV_WGRAD, zero=P1 * C)
            epi = ops.make_epi()
            ws_side = ops.workspace(ops._SPLITK_WS, dev)
            lib.ea_gemm_conv(ctypes.byref(geo), 0, 0, C, 9 * C, K2, dx2.data_ptr(), C, x1p.data_ptr(), C,
                             dw2.data_ptr(), ops.dt(dw2), 9 * C, ctypes.byref(epi), ws_side.data_ptr(),
                             ws_side.numel(), ops.stream())
            ops.permute3(dw2, b.g("conv.2.weight"), C, 9, C, accumulate=True)  # (Co,9,Ci) -> (Co,Ci,9)
        # input gradient per parity class (a, e): sub-pixel decomposition of the transposed
        # conv, ReLU mask of conv1 fused (DACT with aux = x1p).  By default the masked gradient
        # stays on chip: each tile's epilogue multiplies it by conv1's input patches
        # (ea_gemm_conv_w1), so dx1 is never written and conv1's weight / bias gradients are
        # the sum of per-tile partials
        ws = ops.workspace(ops._SPLITK_WS, dev)
        fuse = FUSE_CONV1_WGRAD
        kmaj = DGRAD_KMAJOR and fuse and pos1 is not None and MERGED_DGRAD
        if kmaj:  # W2k: (Co, Ci*9) -> (Ci*9, Co), every output channel's K = (tap, co) row dense
            w2t = empty(C, 9 * C, dtype=cd, device=dev)
            ops.permute3(b.f("conv.2.weight"), w2t, 1, C, 9 * C)
        else:
            w2t = empty(9, C, C, dtype=cd, device=dev)  # tap-major: every tap's (co, ci) block dense
            ops.permute3(b.f("conv.2.weight"), w2t, 1, C * C, 9)  # (Co,Ci,9) -> (9,Co,Ci)
        if fuse:
            _, _, _, rows_all = phase_geo(B, T1, F1, T2, F2, C, CONV_DGRAD)
            part = empty(sum((r + 255) // 256 for r in rows_all) * 10 * C, device=dev)
            tile0 = 0
        else:
            dx1p = empty(P1, C, dtype=cd, device=dev)
        if fuse and pos1 is not None and MERGED_DGRAD:
            # the four parity classes in one launch, longest K first (ea_gemm_conv_w1b_all)
            geo, _, _, _ = phase_geo(B, T1, F1, T2, F2, C, CONV_DGRAD, zero=P2 * C)
            epi = ops.make_epi(EPI_DACT, act=ACT_RELU)
            lib.ea_gemm_conv_w1b_all(ctypes.byref(geo), C, dx2.data_ptr(), C, w2t.data_ptr(), 9 * C if kmaj else C,
                                     ctypes.byref(epi),
                                     feats.data_ptr(), T, Fin, part.data_ptr(), pos1.data_ptr(), ops.stream())
            tile0 = sum((r + 255) // 256 for r in rows_all if r)
        else:
            for a in (0, 1):
                for e in (0, 1):
                    geo, nI, nJ, rows = phase_geo(B, T1, F1, T2, F2, C, CONV_DGRAD, a=a, e=e, zero=P2 * C)
                    Mc = rows[a * 2 + e]
                    if Mc == 0:
                        continue
                    ntaps = (1 if a else 2) * (1 if e else 2)
                    o = geo.plane[a * 2 + e] // C
                    aux = x1p[o:o + Mc]
                    epi = ops.make_epi(EPI_DACT, act=ACT_RELU, aux=aux)
                    if fuse and pos1 is None:
                        lib.ea_gemm_conv_w1(ctypes.byref(geo), Mc, C, ntaps * C, dx2.data_ptr(), C, w2t.data_ptr(), C,
                                            ctypes.byref(epi), feats.data_ptr(), T, Fin,
                                            part.data_ptr() + 4 * tile0 * 10 * C, ops.stream())
                        tile0 += (Mc + 255) // 256
                    elif fuse:
                        lib.ea_gemm_conv_w1b(ctypes.byref(geo), Mc, C, ntaps * C, dx2.data_ptr(), C, w2t.data_ptr(), C,
                                             ctypes.byref(epi), feats.data_ptr(), T, Fin,
                                             part.data_ptr() + 4 * tile0 * 10 * C, pos1.data_ptr() + o * (C // 8),
                                             ops.stream())
                        tile0 += (Mc + 255) // 256
                    else:
                        lib.ea_gemm_conv(ctypes.byref(geo), 1, 0, Mc, C, ntaps * C, dx2.data_ptr(), C, w2t.data_ptr(),
                                         C, dx1p[o:o + Mc].data_ptr(), ops.dt(dx1p), C, ctypes.byref(epi),
                                         ws.data_ptr(), ws.numel(), ops.stream())
        if fuse:
            lib.ea_conv1_wgrad_reduce(tile0, C, part.data_ptr(), b.g("conv.0.weight").data_ptr(),
                                      b.g("conv.0.bias").data_ptr(), ops.stream())
        else:
            with ops.wgrad(dx1p, feats, launches=True):
                w, wn = ops._ws(dev, 1024 * 10 * C)
                lib.ea_conv1_wgrad(B, T, Fin, C, feats.data_ptr(), dx1p.data_ptr(), ops.dt(dx1p),
                                   b.g("conv.0.weight").data_ptr(), b.g("conv.0.bias").data_ptr(), w, wn, ops.stream())
        ops.grad_ready(b)
        return None, None, None, None, None

    @staticmethod
    def backward(ctx, dy):
        if ctx.implicit:
            return SubsampleFn._backward_implicit(ctx, dy)
        m = ctx.m
        b = m._b
        cd = b.cd
        B, T, Fin, T1, F1, T2, F2, p, seed = ctx.meta
        col1, x1, col2, w2, x2, wl = ctx.save
        ctx.save = None
        C = m.odim
        dev = dy.device
        dv = empty(B * T2, C, dtype=cd, device=dev)
        ops.scale_dropout_colsum(dy.reshape(B * T2, C).contiguous(), dv, b.g("out.0.bias"), scale=m.out[1].xscale,
                                 p=p, seed=seed)
        x2r = x2.view(B * T2, F2 * C)
        with ops.wgrad(dv, x2):
            dwl = empty(C, F2 * C, device=dev)
            gw = b.g("out.0.weight")
            ops.linear_dw(dv, x2r, dwl, accumulate=False,  # then (d,F2,C) -> (d,C,F2) into the arena
                          post=lambda: ops.permute3(dwl, gw, C, F2, C, accumulate=True))
        dx2 = empty(B * T2, F2 * C, dtype=cd, device=dev)
        ops.linear_dx(dv, wl, dx2, epi=ops.make_epi(EPI_DACT, act=ACT_RELU, aux=x2r))
        dx2 = dx2.view(-1, C)
        with ops.wgrad(dx2, col2):
            ops.colsum(dx2, b.g("conv.2.bias"))
            dw2 = empty(C, 9 * C, device=dev)
            g2 = b.g("conv.2.weight")
            ops.linear_dw(dx2, col2, dw2, accumulate=False,  # then (Co,9,Ci) -> (Co,Ci,9) into the arena
                          post=lambda: ops.permute3(dw2, g2, C, 9, C, accumulate=True))
        dcol2 = empty(*col2.shape, dtype=cd, device=dev)
        ops.linear_dx(dx2, w2, dcol2)
        del col2
        dx1 = empty(*x1.shape, dtype=cd, device=dev)
        lib.ea_col2im_conv2(B, T1, F1, C, dcol2.data_ptr(), ops.dt(dcol2), x1.data_ptr(), dx1.data_ptr(),
                            ops.dt(dx1), ops.stream())
        del dcol2
        with ops.wgrad(dx1, col1, launches=True):
            ops.colsum(dx1, b.g("conv.0.bias"))
            ops.gemm(dx1, col1, b.g("conv.0.weight", shape=(C, 9)), M=C, N=9, K=dx1.shape[0],
                     a_kmajor=0, b_kmajor=0, lda=C, ldb=16, ldc=9, epi=ops.make_epi(beta=1.0))
        ops.grad_ready(b)
        return None, None, None, None, None
