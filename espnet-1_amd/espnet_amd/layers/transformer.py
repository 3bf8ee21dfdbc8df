"""Transformer encoder block — espnet/nets/pytorch_backend/transformer/encoder_layer.py:
EncoderLayer (normalize_before=True, concat_after=False, no stochastic depth):

    x = x + dropout(self_attn(norm1(x), mask))          (encoder_layer.py:98-112)
    x = x + dropout(feed_forward(norm2(x)))             (:114-118)

with MultiHeadedAttention (attention.py:15-111, key-padding mask) and the ReLU
PositionwiseFeedForward (positionwise_feed_forward.py:22-32).  One autograd node per
block (`TransformerBlockFn`) over the same HIP kernels as the decoder's self-attention
and FFN: fused q/k/v GEMM, fused flash attention (bf16, d_k = 64) or the GEMM + softmax
path, GEMM epilogues for bias / ReLU / dropout / residual.
"""
from __future__ import annotations

import math

import torch
from torch import nn

from .common import (ACT_RELU, EPI_ACT, EPI_DACT, EPI_RESID, Bound, empty, ln_bwd, ln_fwd, ops, site_dv,
                     site_seed)
from .conformer import LayerNorm
from .decoder import _mha_bwd, _mha_fwd


class TransformerEncoderLayer(nn.Module):
    """transformer/encoder_layer.py:34-55 parameter set (self_attn, feed_forward, norm1, norm2)."""

    def __init__(self, size, self_attn, feed_forward, dropout_rate, normalize_before=True, concat_after=False,
                 stochastic_depth_rate=0.0):
        super().__init__()
        if not normalize_before or concat_after or stochastic_depth_rate > 0:
            raise NotImplementedError("only normalize_before=True, concat_after=False, "
                                      "stochastic_depth_rate=0 are implemented")
        self.self_attn = self_attn
        self.feed_forward = feed_forward
        self.norm1 = LayerNorm(size)
        self.norm2 = LayerNorm(size)
        self.size = size
        self.dropout_rate = dropout_rate
        self.layer_idx = 0
        self._b = None

    def bind(self, arena, prefix, cd):
        self._b = Bound(arena, prefix, cd)

    @staticmethod
    def arena_groups(prefix):
        a = prefix + "self_attn."
        return [[a + "linear_q.weight", a + "linear_k.weight", a + "linear_v.weight"],
                [a + "linear_q.bias", a + "linear_k.bias", a + "linear_v.bias"]]

    def forward(self, x, olens, seed):
        return TransformerBlockFn.apply(x, olens, self, seed, self.training)


_QKV_W = ("self_attn.linear_q.weight", "self_attn.linear_k.weight", "self_attn.linear_v.weight")
_QKV_B = ("self_attn.linear_q.bias", "self_attn.linear_k.bias", "self_attn.linear_v.bias")


class TransformerBlockFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, olens, L: TransformerEncoderLayer, seed, training):
        b = L._b
        cd = b.cd
        B, T, d = x.shape
        N = B * T
        dev = x.device
        H = L.self_attn.h
        dk = d // H
        p = L.dropout_rate if training else 0.0
        pa = L.self_attn.dropout_rate if training else 0.0
        p_ff = L.feed_forward.dropout_rate if training else 0.0
        sd = lambda s: site_seed(seed, 50 + L.layer_idx, s)  # noqa: E731
        scale = 1.0 / math.sqrt(dk)
        x0 = x.reshape(N, d)
        # ---- self-attention
        xn1, mu1, rs1 = ln_fwd(x0, b, "norm1", cd)
        qkv = empty(N, 3 * d, dtype=cd, device=dev)
        ops.linear(xn1, b.w(*_QKV_W, shape=(3 * d, d)), qkv, epi=ops.make_epi(bias=b.f(*_QKV_B, shape=(3 * d,))))
        O, st = _mha_fwd(qkv, qkv[:, d:], qkv[:, 2 * d:], B=B, H=H, T1=T, T2=T, dk=dk, ldq=3 * d, ldk=3 * d,
                         ldv=3 * d, klen=olens, causal=getattr(L, "causal", False), scale=scale, p=pa, seed=sd(1), cd=cd)
        x1 = empty(N, d, device=dev)
        ops.linear(O, b.w("self_attn.linear_out.weight"), x1,
                   epi=ops.make_epi(EPI_RESID, bias=b.f("self_attn.linear_out.bias"), resid=x0, drop_p=p,
                                    seed=sd(2)))
        # ---- feed-forward (ReLU)
        xn2, mu2, rs2 = ln_fwd(x1, b, "norm2", cd)
        Fh = L.feed_forward.w_1.out_features
        h = empty(N, Fh, dtype=cd, device=dev)
        a = empty(N, Fh, dtype=cd, device=dev)
        ops.linear(xn2, b.w("feed_forward.w_1.weight"), a,
                   epi=ops.make_epi(EPI_ACT, bias=b.f("feed_forward.w_1.bias"), act=ACT_RELU, aux=h, drop_p=p_ff,
                                    seed=sd(3)))
        x2 = empty(N, d, device=dev)
        ops.linear(a, b.w("feed_forward.w_2.weight"), x2,
                   epi=ops.make_epi(EPI_RESID, bias=b.f("feed_forward.w_2.bias"), resid=x1, drop_p=p, seed=sd(4)))
        ctx.L = L
        ctx.meta = (B, T, d, H, dk, p, pa, p_ff, seed, scale)
        ctx.save = (x0, x1, (xn1, mu1, rs1, qkv, O, st), (xn2, mu2, rs2, h, a), olens)
        return x2.view(B, T, d)

    @staticmethod
    def backward(ctx, dout):
        L = ctx.L
        b = L._b
        cd = b.cd
        B, T, d, H, dk, p, pa, p_ff, seed, scale = ctx.meta
        x0, x1, s_att, s_ff, olens = ctx.save
        ctx.save = None
        sd = lambda s: site_seed(seed, 50 + L.layer_idx, s)  # noqa: E731
        N = B * T
        dev = dout.device
        dx = dout.reshape(N, d).contiguous().clone()
        # ---- feed-forward
        xn2, mu2, rs2, h, a = s_ff
        dv = site_dv(dx, None, b.g("feed_forward.w_2.bias"), 1.0, p, sd(4), cd)
        with ops.wgrad(dv, a):
            ops.linear_dw(dv, a, b.g("feed_forward.w_2.weight"), accumulate=True)
        dh = empty(*h.shape, dtype=cd, device=dev)
        ops.linear_dx(dv, b.w("feed_forward.w_2.weight"), dh,
                      epi=ops.make_epi(EPI_DACT, act=ACT_RELU, aux=h, drop_p=p_ff, seed=sd(3)))
        with ops.wgrad(dh, xn2):
            ops.colsum(dh, b.g("feed_forward.w_1.bias"))
            ops.linear_dw(dh, xn2, b.g("feed_forward.w_1.weight"), accumulate=True)
        dxn = empty(N, d, dtype=cd, device=dev)
        ops.linear_dx(dh, b.w("feed_forward.w_1.weight"), dxn)
        ln_bwd(dxn, x1, b, "norm2", mu2, rs2, dx, accumulate=True)
        # ---- self-attention
        xn1, mu1, rs1, qkv, O, st = s_att
        dv = site_dv(dx, None, b.g("self_attn.linear_out.bias"), 1.0, p, sd(2), cd)
        with ops.wgrad(dv, O):
            ops.linear_dw(dv, O, b.g("self_attn.linear_out.weight"), accumulate=True)
        dO = empty(N, d, dtype=cd, device=dev)
        ops.linear_dx(dv, b.w("self_attn.linear_out.weight"), dO)
        dqkv = empty(N, 3 * d, dtype=cd, device=dev)
        _mha_bwd(st, dO, qkv, qkv[:, d:], qkv[:, 2 * d:], B=B, H=H, T1=T, T2=T, dk=dk, ldq=3 * d, ldk=3 * d,
                 ldv=3 * d, klen=olens, causal=getattr(L, "causal", False), scale=scale, p=pa, seed=sd(1), cd=cd, dq=dqkv, lddq=3 * d,
                 dk_=dqkv[:, d:], lddk=3 * d, dv=dqkv[:, 2 * d:], lddv=3 * d)
        with ops.wgrad(dqkv, xn1):
            ops.colsum(dqkv, b.g(*_QKV_B, shape=(3 * d,)))
            ops.linear_dw(dqkv, xn1, b.g(*_QKV_W, shape=(3 * d, d)), accumulate=True)
        dxn = empty(N, d, dtype=cd, device=dev)
        ops.linear_dx(dqkv, b.w(*_QKV_W, shape=(3 * d, d)), dxn)
        ln_bwd(dxn, x0, b, "norm1", mu1, rs1, dx, accumulate=True)
        ops.grad_ready(b)
        return dx.view(B, T, d), None, None, None, None
