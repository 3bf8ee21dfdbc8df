"""Conformer encoder block — espnet/nets/pytorch_backend/conformer/encoder_layer.py:79-179
(normalize_before=True, concat_after=False, macaron FFN, rel-pos MHSA, conv module).

Parameter holders keep the reference's attribute names, constructor order and torch
default initialisation (so the same seed gives the same weights and the same state_dict
keys); the computation is `ConformerBlockFn`: one autograd node per block running the
block's HIP kernels forward and its hand-written backward.

Data layout (channel-last, token-major): x (B*T, d) f32 residual stream; GEMM operands in
the compute dtype cd (f32, or bf16 under AMP); the fused qkv (B*T, 3d) keeps heads as
column blocks so attention reads q/k/v with strides, no transposes.
"""
from __future__ import annotations

import ctypes
import os

import torch
from torch import nn

from .common import (ACT_SWISH, EPI_ACT, EPI_DACT, EPI_RESID, EPI_STORE, F32, Bound, attn_bwd, attn_dmask, dbd_layout,
                     attn_fused_bwd, attn_fwd, empty, fused_attn_ok, lib, ln_bwd, ln_fwd, math, ops, ptr, rup,
                     site_seed, dv_buf, drop_arg, site_dv)


# ----------------------------------------------------------------------------- holders

# the GLU backward fused into the depthwise conv's backward kernel (ea_dwconv_glu_bwd: the
# same arithmetic without the f32 dglu round trip; EA_FUSE_DW_GLU=0: the two-kernel path)
FUSE_DW_GLU = os.environ.get("EA_FUSE_DW_GLU", "1") != "0"
# the depthwise conv's forward and backward read glu(g2) from the bf16 pointwise-conv output
# instead of a stored f32 GLU activation (ea_dwconv_fwd_glu / ea_dwconv_glu_bwd with x = NULL;
# EA_GLU_IN_CONV=0: glu_fwd + the stored activation)
GLU_IN_CONV = os.environ.get("EA_GLU_IN_CONV", "1") != "0"
# with it, the depthwise conv forward also writes the BatchNorm's batch-statistics partials
# (ea_dwconv_fwd_glu_stats + ea_batchnorm_fwd_parts; EA_BN_STATS_IN_CONV=0: a statistics pass
# over y; measured 17.83-17.88 -> 17.73-17.76 ms per C3 step)
BN_STATS_IN_CONV = os.environ.get("EA_BN_STATS_IN_CONV", "1") != "0"


def _glu_in_conv(K, g2, d):
    return (GLU_IN_CONV and FUSE_DW_GLU and K in (3, 5, 7, 15, 31)
            and g2.dtype == torch.bfloat16 and d % 4 == 0 and g2.data_ptr() % 8 == 0 and torch.cuda.is_available())

class PositionwiseFeedForward(nn.Module):
    """positionwise_feed_forward.py:12-32 (w_2(dropout(act(w_1 x))))."""

    def __init__(self, idim, hidden_units, dropout_rate, activation="swish"):
        super().__init__()
        self.w_1 = nn.Linear(idim, hidden_units)
        self.w_2 = nn.Linear(hidden_units, idim)
        self.dropout_rate = dropout_rate
        self.activation = activation


class MultiHeadedAttention(nn.Module):
    """transformer/attention.py:15-37 parameter set."""

    def __init__(self, n_head, n_feat, dropout_rate):
        super().__init__()
        assert n_feat % n_head == 0
        self.d_k = n_feat // n_head
        self.h = n_head
        self.linear_q = nn.Linear(n_feat, n_feat)
        self.linear_k = nn.Linear(n_feat, n_feat)
        self.linear_v = nn.Linear(n_feat, n_feat)
        self.linear_out = nn.Linear(n_feat, n_feat)
        self.dropout_rate = dropout_rate


class RelPositionMultiHeadedAttention(MultiHeadedAttention):
    """transformer/attention.py:209-235 parameter set (linear_pos, pos_bias_u/v)."""

    def __init__(self, n_head, n_feat, dropout_rate, zero_triu=False):
        super().__init__(n_head, n_feat, dropout_rate)
        if zero_triu:
            raise NotImplementedError("zero_triu=True is not on the ASR hot path")
        self.linear_pos = nn.Linear(n_feat, n_feat, bias=False)
        self.pos_bias_u = nn.Parameter(torch.Tensor(self.h, self.d_k))
        self.pos_bias_v = nn.Parameter(torch.Tensor(self.h, self.d_k))
        torch.nn.init.xavier_uniform_(self.pos_bias_u)
        torch.nn.init.xavier_uniform_(self.pos_bias_v)


class ConvolutionModule(nn.Module):
    """conformer/convolution.py:13-54 parameter set."""

    def __init__(self, channels, kernel_size, activation="swish", bias=True):
        super().__init__()
        assert (kernel_size - 1) % 2 == 0
        self.pointwise_conv1 = nn.Conv1d(channels, 2 * channels, 1, 1, 0, bias=bias)
        self.depthwise_conv = nn.Conv1d(channels, channels, kernel_size, 1, (kernel_size - 1) // 2,
                                        groups=channels, bias=bias)
        self.norm = nn.BatchNorm1d(channels)
        self.pointwise_conv2 = nn.Conv1d(channels, channels, 1, 1, 0, bias=bias)
        self.kernel_size = kernel_size


def LayerNorm(n):  # transformer/layer_norm.py:12 (eps=1e-12 applied by the kernels)
    return nn.LayerNorm(n, eps=1e-12)


class EncoderLayer(nn.Module):
    """conformer/encoder_layer.py:43-77 parameter set + HIP forward."""

    def __init__(self, size, self_attn, feed_forward, feed_forward_macaron, conv_module,
                 dropout_rate, normalize_before=True, concat_after=False, stochastic_depth_rate=0.0):
        super().__init__()
        if not normalize_before or concat_after or stochastic_depth_rate > 0:
            raise NotImplementedError("only normalize_before=True, concat_after=False, "
                                      "stochastic_depth_rate=0 (the ASR recipes) are implemented")
        if conv_module is None:
            raise NotImplementedError("use_cnn_module=False is not on the hot path")
        self.self_attn = self_attn
        self.feed_forward = feed_forward
        self.feed_forward_macaron = feed_forward_macaron
        self.conv_module = conv_module
        self.norm_ff = LayerNorm(size)
        self.norm_mha = LayerNorm(size)
        if feed_forward_macaron is not None:
            self.norm_ff_macaron = LayerNorm(size)
            self.ff_scale = 0.5
        else:
            self.ff_scale = 1.0
        self.norm_conv = LayerNorm(size)
        self.norm_final = LayerNorm(size)
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

    def forward(self, x, pos_emb, olens, seed):
        return ConformerBlockFn.apply(x, pos_emb, olens, self, seed, self.training)


# ----------------------------------------------------------------------------- forward pieces
def _ffn_fwd(L, b, x_in, pre, ln_name, p, seed_in, seed_out):
    cd = b.cd
    N, d = x_in.shape
    Fh = L.feed_forward.w_1.out_features
    xn, mu, rs = ln_fwd(x_in, b, ln_name, cd)
    h = empty(N, Fh, dtype=cd, device=x_in.device)
    a = empty(N, Fh, dtype=cd, device=x_in.device)
    ops.linear(xn, b.w(pre + ".w_1.weight"), a,
               epi=ops.make_epi(EPI_ACT, bias=b.f(pre + ".w_1.bias"), act=ACT_SWISH, aux=h,
                                drop_p=p, seed=seed_in))
    x_out = empty(N, d, device=x_in.device)
    ops.linear(a, b.w(pre + ".w_2.weight"), x_out,
               epi=ops.make_epi(EPI_RESID, bias=b.f(pre + ".w_2.bias"), resid=x_in,
                                rscale=L.ff_scale, drop_p=p, seed=seed_out))
    return x_out, (xn, mu, rs, h, a)


def _ffn_bwd(L, b, dx, x_in, saved, pre, ln_name, p, seed_in, seed_out, dv_in=None, next_drop=None):
    """dx: f32 (N,d) grad of the sub-block output; updated in place to grad of x_in.  dv_in: this
    site's dv when already written; next_drop: the following site's (dv, scale, p, seed) for the
    LayerNorm backward to write."""
    cd = b.cd
    xn, mu, rs, h, a = saved
    N, d = dx.shape
    dv = site_dv(dx, dv_in, b.g(pre + ".w_2.bias"), L.ff_scale, p, seed_out, cd)
    with ops.wgrad(dv, a):
        ops.linear_dw(dv, a, b.g(pre + ".w_2.weight"), accumulate=True)
    dh = empty(*h.shape, dtype=cd, device=dx.device)
    ops.linear_dx(dv, b.w(pre + ".w_2.weight"), dh,
                  epi=ops.make_epi(EPI_DACT, act=ACT_SWISH, aux=h, drop_p=p, seed=seed_in))
    with ops.wgrad(dh, xn):
        ops.colsum(dh, b.g(pre + ".w_1.bias"))
        ops.linear_dw(dh, xn, b.g(pre + ".w_1.weight"), accumulate=True)
    dxn = empty(N, d, dtype=cd, device=dx.device)
    ops.linear_dx(dh, b.w(pre + ".w_1.weight"), dxn)
    ln_bwd(dxn, x_in, b, ln_name, mu, rs, dx, accumulate=True, drop=next_drop)


class ConformerBlockFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, pos, olens, L: EncoderLayer, seed, training):
        b = L._b
        cd = b.cd
        B, T, d = x.shape
        N = B * T
        dev = x.device
        H = L.self_attn.h
        dk = d // H
        P2 = 2 * T - 1
        p = L.dropout_rate if training else 0.0
        pa = L.self_attn.dropout_rate if training else 0.0
        li = L.layer_idx
        sd = lambda s: site_seed(seed, li, s)  # noqa: E731
        x0 = x.reshape(N, d)
        # ---- macaron FFN  (encoder_layer.py:115-123)
        x1, s_ff1 = _ffn_fwd(L, b, x0, "feed_forward_macaron", "norm_ff_macaron", p, sd(1), sd(2))
        # ---- rel-pos MHSA (encoder_layer.py:126-149, attention.py:262-305)
        xn2, mu2, rs2 = ln_fwd(x1, b, "norm_mha", cd)
        A = "self_attn."
        qkv = empty(N, 3 * d, dtype=cd, device=dev)
        ops.linear(xn2, b.w(A + "linear_q.weight", A + "linear_k.weight", A + "linear_v.weight",
                            shape=(3 * d, d)), qkv,
                   epi=ops.make_epi(bias=b.f(A + "linear_q.bias", A + "linear_k.bias",
                                             A + "linear_v.bias", shape=(3 * d,))))
        pp = empty(P2, d, dtype=cd, device=dev)
        ops.linear(pos, b.w(A + "linear_pos.weight"), pp)
        scale = 1.0 / math.sqrt(dk)
        if fused_attn_ok(cd, dk, T, T):
            # one kernel: (q+u)k^T + rel_shift((q+v)p^T), mask, softmax, dropout, @v
            O = empty(N, d, dtype=cd, device=dev)
            lse = empty(B * H * T, device=dev)
            dmask, ldm = attn_dmask(B * H * T, T, pa, dev)
            lib.ea_attn_fused_fwd2(B, H, T, T, dk, qkv.data_ptr(), 3 * d, qkv[:, d:].data_ptr(), 3 * d,
                                   qkv[:, 2 * d:].data_ptr(), 3 * d, b.f(A + "pos_bias_u").data_ptr(),
                                   b.f(A + "pos_bias_v").data_ptr(), pp.data_ptr(), d, olens.data_ptr(), 0,
                                   scale, float(pa), sd(3), O.data_ptr(), d, lse.data_ptr(), ptr(dmask), ldm,
                                   ops.stream())
            ldT = 0
            s_core = ("fused", lse, dmask, ldm)
        else:
            qu = empty(N, d, dtype=cd, device=dev)
            qv = empty(N, d, dtype=cd, device=dev)
            lib.ea_add_pos_bias(N, H, dk, qkv.data_ptr(), 3 * d, b.f(A + "pos_bias_u").data_ptr(),
                                b.f(A + "pos_bias_v").data_ptr(), qu.data_ptr(), qv.data_ptr(),
                                ops.dt(qu), ops.stream())
            ldbd = rup(P2, 8)
            bd = empty(H * B * T * ldbd, device=dev)
            ops.gemm(qv, pp, bd, M=T, N=P2, K=dk, a_kmajor=1, b_kmajor=1, lda=d, ldb=d, ldc=ldbd,
                     batch=B, nh=H, sA=(T * d, dk), sB=(0, dk), sC=(T * ldbd, B * T * ldbd), splitk=False)
            O, P, Pd, ldT = attn_fwd(qu, qkv[:, d:], qkv[:, 2 * d:], B=B, H=H, T1=T, T2=T, dk=dk,
                                     ldq=d, ldk=3 * d, ldv=3 * d, klen=olens, causal=False, scale=scale,
                                     p=pa, seed=sd(3), cd=cd, bd=bd, ldbd=ldbd)
            del bd
            s_core = ("unfused", qu, qv, P, Pd)
        x2 = empty(N, d, device=dev)
        ops.linear(O, b.w(A + "linear_out.weight"), x2,
                   epi=ops.make_epi(EPI_RESID, bias=b.f(A + "linear_out.bias"), resid=x1,
                                    drop_p=p, seed=sd(4)))
        # ---- conv module (encoder_layer.py:152-158, convolution.py:56-79)
        C = "conv_module."
        K = L.conv_module.kernel_size
        xn3, mu3, rs3 = ln_fwd(x2, b, "norm_conv", cd)
        g2 = empty(N, 2 * d, dtype=cd, device=dev)
        ops.linear(xn3, b.w(C + "pointwise_conv1.weight", shape=(2 * d, d)), g2,
                   epi=ops.make_epi(bias=b.f(C + "pointwise_conv1.bias")))
        y = empty(N, d, device=dev)
        bn_part = None
        if _glu_in_conv(K, g2, d):
            # the depthwise conv reads glu(g2) straight from the pointwise conv's bf16 output; the
            # f32 GLU activation is neither stored nor re-read (the backward recomputes it too)
            glu = None
            if training and BN_STATS_IN_CONV:
                # ... and writes the BatchNorm's batch-statistics partials of its tiles
                npart = ctypes.c_int(0)
                lib.ea_dwconv_stats_parts(B, T, ctypes.addressof(npart))
                bn_part = (empty(npart.value * 2 * d, device=dev), npart.value)
                lib.ea_dwconv_fwd_glu_stats(B, T, d, K, g2.data_ptr(), b.f(C + "depthwise_conv.weight").data_ptr(),
                                            b.f(C + "depthwise_conv.bias").data_ptr(), y.data_ptr(),
                                            bn_part[0].data_ptr(), ops.stream())
            else:
                lib.ea_dwconv_fwd_glu(B, T, d, K, g2.data_ptr(), b.f(C + "depthwise_conv.weight").data_ptr(),
                                      b.f(C + "depthwise_conv.bias").data_ptr(), y.data_ptr(), ops.stream())
        else:
            glu = empty(N, d, device=dev)
            lib.ea_glu_fwd(N, d, g2.data_ptr(), ops.dt(g2), glu.data_ptr(), 0, ops.stream())
            lib.ea_dwconv_fwd(B, T, d, K, glu.data_ptr(), b.f(C + "depthwise_conv.weight").data_ptr(),
                              b.f(C + "depthwise_conv.bias").data_ptr(), y.data_ptr(), ops.stream())
        z = empty(N, d, dtype=cd, device=dev)
        bn_mean = empty(d, device=dev)
        bn_rstd = empty(d, device=dev)
        bn = L.conv_module.norm
        if bn_part is not None:
            lib.ea_batchnorm_fwd_parts(N, d, y.data_ptr(), bn_part[0].data_ptr(), bn_part[1],
                                       b.f(C + "depthwise_conv.bias").data_ptr(), b.f(C + "norm.weight").data_ptr(),
                                       b.f(C + "norm.bias").data_ptr(), float(bn.eps), float(bn.momentum),
                                       bn_mean.data_ptr(), bn_rstd.data_ptr(), ops.ptr(bn.running_mean),
                                       ops.ptr(bn.running_var), ops.ptr(bn.num_batches_tracked), ACT_SWISH,
                                       z.data_ptr(), ops.dt(z), ops.stream())
        else:
            ops.batchnorm_fwd(y, b.f(C + "norm.weight"), b.f(C + "norm.bias"), bn_mean, bn_rstd,
                              bn.running_mean, bn.running_var, bn.num_batches_tracked, z,
                              training, ACT_SWISH, eps=bn.eps, momentum=bn.momentum)
        x3 = empty(N, d, device=dev)
        ops.linear(z, b.w(C + "pointwise_conv2.weight", shape=(d, d)), x3,
                   epi=ops.make_epi(EPI_RESID, bias=b.f(C + "pointwise_conv2.bias"), resid=x2,
                                    drop_p=p, seed=sd(5)))
        # ---- FFN (encoder_layer.py:161-168) + norm_final (:170-171)
        x4, s_ff2 = _ffn_fwd(L, b, x3, "feed_forward", "norm_ff", p, sd(6), sd(7))
        out, mu5, rs5 = ln_fwd(x4, b, "norm_final", F32)
        ctx.L = L
        ctx.meta = (B, T, d, H, dk, p, pa, seed, scale, ldT)
        ctx.save = (x0, x1, x2, x3, x4, s_ff1, (xn2, mu2, rs2, qkv, pp, O, s_core),
                    (xn3, mu3, rs3, g2, glu, y, z, bn_mean, bn_rstd), s_ff2, (mu5, rs5), pos, olens)
        return out.view(B, T, d)

    @staticmethod
    def backward(ctx, dout):
        L = ctx.L
        b = L._b
        cd = b.cd
        B, T, d, H, dk, p, pa, seed, scale, ldT = ctx.meta
        (x0, x1, x2, x3, x4, s_ff1, s_att, s_conv, s_ff2, (mu5, rs5), pos, olens) = ctx.save
        ctx.save = None
        li = L.layer_idx
        sd = lambda s: site_seed(seed, li, s)  # noqa: E731
        N = B * T
        dev = dout.device
        P2 = 2 * T - 1
        dx = empty(N, d, device=dev)
        dv_ff2 = dv_buf(N, d, cd, dev)
        ln_bwd(dout.reshape(N, d).contiguous(), x4, b, "norm_final", mu5, rs5, dx, accumulate=False,
               drop=drop_arg(dv_ff2, L.ff_scale, p, sd(7), b.g("feed_forward.w_2.bias")))
        # ---- FFN
        dv_conv = dv_buf(N, d, cd, dev)
        _ffn_bwd(L, b, dx, x3, s_ff2, "feed_forward", "norm_ff", p, sd(6), sd(7), dv_in=dv_ff2,
                 next_drop=drop_arg(dv_conv, 1.0, p, sd(5), b.g("conv_module.pointwise_conv2.bias")))
        # ---- conv module
        C = "conv_module."
        K = L.conv_module.kernel_size
        xn3, mu3, rs3, g2, glu, y, z, bn_mean, bn_rstd = s_conv
        dv = site_dv(dx, dv_conv, b.g(C + "pointwise_conv2.bias"), 1.0, p, sd(5), cd)
        with ops.wgrad(dv, z):
            ops.linear_dw(dv, z, b.g(C + "pointwise_conv2.weight", shape=(d, d)), accumulate=True)
        dz = empty(N, d, dtype=cd, device=dev)
        ops.linear_dx(dv, b.w(C + "pointwise_conv2.weight", shape=(d, d)), dz)
        dy = empty(N, d, device=dev)
        ops.batchnorm_bwd(dz, y, bn_mean, bn_rstd, b.f(C + "norm.weight"), b.f(C + "norm.bias"),
                          ACT_SWISH, dy, b.g(C + "norm.weight"), b.g(C + "norm.bias"))
        dg2 = empty(N, 2 * d, dtype=cd, device=dev)
        fuse = FUSE_DW_GLU and K in (3, 5, 7, 15, 31) and g2.dtype == torch.bfloat16
        if fuse:
            # the GLU backward inside the depthwise conv's input-gradient store (no f32 dglu)
            w, wn = ops._ws(dev, B * ((T + 31) // 32) * d * (K + 1) + 1024)
            lib.ea_dwconv_glu_bwd(B, T, d, K, ops.ptr(glu), b.f(C + "depthwise_conv.weight").data_ptr(),
                                  dy.data_ptr(), g2.data_ptr(), dg2.data_ptr(),
                                  b.g(C + "depthwise_conv.weight").data_ptr(),
                                  b.g(C + "depthwise_conv.bias").data_ptr(), 1, w, wn, ops.stream())
        else:
            if glu is None:  # (forward without the stored activation, backward on the two-kernel path)
                glu = empty(N, d, device=dev)
                lib.ea_glu_fwd(N, d, g2.data_ptr(), ops.dt(g2), glu.data_ptr(), 0, ops.stream())
            dglu = empty(N, d, device=dev)
            w, wn = ops._ws(dev, B * ((T + 31) // 32) * d * (K + 1) + 1024)
            lib.ea_dwconv_bwd(B, T, d, K, glu.data_ptr(), b.f(C + "depthwise_conv.weight").data_ptr(),
                              dy.data_ptr(), dglu.data_ptr(), b.g(C + "depthwise_conv.weight").data_ptr(),
                              b.g(C + "depthwise_conv.bias").data_ptr(), 1, w, wn, ops.stream())
            lib.ea_glu_bwd(N, d, g2.data_ptr(), ops.dt(g2), dglu.data_ptr(), dg2.data_ptr(), ops.stream())
        with ops.wgrad(dg2, xn3):
            ops.colsum(dg2, b.g(C + "pointwise_conv1.bias"))
            ops.linear_dw(dg2, xn3, b.g(C + "pointwise_conv1.weight", shape=(2 * d, d)), accumulate=True)
        dxn3 = empty(N, d, dtype=cd, device=dev)
        ops.linear_dx(dg2, b.w(C + "pointwise_conv1.weight", shape=(2 * d, d)), dxn3)
        dv_att = dv_buf(N, d, cd, dev)
        ln_bwd(dxn3, x2, b, "norm_conv", mu3, rs3, dx, accumulate=True,
               drop=drop_arg(dv_att, 1.0, p, sd(4), b.g("self_attn.linear_out.bias")))
        # ---- rel-pos MHSA
        A = "self_attn."
        xn2, mu2, rs2, qkv, pp, O, s_core = s_att
        dv = site_dv(dx, dv_att, b.g(A + "linear_out.bias"), 1.0, p, sd(4), cd)
        with ops.wgrad(dv, O):
            ops.linear_dw(dv, O, b.g(A + "linear_out.weight"), accumulate=True)
        dO = empty(N, d, dtype=cd, device=dev)
        ops.linear_dx(dv, b.w(A + "linear_out.weight"), dO)
        dqkv = empty(N, 3 * d, dtype=cd, device=dev)
        ldbd, shift = rup(P2, 8), 0
        if s_core[0] == "fused":
            # dq includes the q+v path (dBD.p, in-kernel); dbd rows written in full, in the
            # pipelined dQ pass's shifted layout (logical column r at r + shift); pos_bias_u /
            # pos_bias_v gradients from per-block column sums of the two dq terms
            _, lse, dmask, ldm = s_core
            shift, ldbd = dbd_layout(T)
            dbd = empty(H * B * T * ldbd, dtype=cd, device=dev)
            qv = empty(N, d, dtype=cd, device=dev)  # q + v, for the linear_pos weight gradient
            nqb = (T + 63) // 64
            part = empty(2 * B * nqb * d, device=dev)
            attn_fused_bwd(B=B, H=H, T1=T, T2=T, q=qkv, ldq=3 * d, k=qkv[:, d:], ldk=3 * d, v=qkv[:, 2 * d:],
                           ldv=3 * d, bu=b.f(A + "pos_bias_u"), bv=b.f(A + "pos_bias_v"), pp=pp, ldp=d,
                           klen=olens, causal=False, scale=scale, p=pa, seed=sd(3), O=O, ldo=d, lse=lse, dO=dO,
                           lddo=d, dq=dqkv, lddq=3 * d, dk=dqkv[:, d:], lddk=3 * d, dv=dqkv[:, 2 * d:],
                           lddv=3 * d, dbd=dbd, ldbd=ldbd, part=part, ldpart=d, qv_out=qv, ldqv=d, dmask=dmask,
                           ldm=ldm, flags=1 | 2)
            ops.reduce_rows(part[:B * nqb * d], B * nqb, d, d, b.g(A + "pos_bias_u", shape=(d,)))
            ops.reduce_rows(part[B * nqb * d:], B * nqb, d, d, b.g(A + "pos_bias_v", shape=(d,)))
        else:
            _, qu, qv, P, Pd = s_core
            dbd = empty(H * B * T * ldbd, dtype=cd, device=dev)
            attn_bwd(dO, qu, qkv[:, d:], qkv[:, 2 * d:], P, Pd, ldT, B=B, H=H, T1=T, T2=T, dk=dk,
                     ldq=d, ldk=3 * d, ldv=3 * d, scale=scale, p=pa, seed=sd(3), cd=cd,
                     dq=dqkv, lddq=3 * d, dk_=dqkv[:, d:], lddk=3 * d, dv=dqkv[:, 2 * d:], lddv=3 * d,
                     dbd=dbd, ldbd=ldbd)
            # q_u = q + u: du = sum dq_u ; q_v = q + v path: dq_v = dBD . p_h, dv_bias = sum dq_v
            dqv = empty(N, d, dtype=cd, device=dev)
            ops.gemm(dbd, pp, dqv, M=T, N=dk, K=P2, a_kmajor=1, b_kmajor=0, lda=ldbd, ldb=d, ldc=d,
                     batch=B, nh=H, sA=(T * ldbd, B * T * ldbd), sB=(0, dk), sC=(T * d, dk), splitk=False)
            # not deferred: dqkv[:, :d] receives dqv in place right below
            ops.colsum(dqkv[:, :d], b.g(A + "pos_bias_u", shape=(d,)), defer=False)
            ops.colsum(dqv, b.g(A + "pos_bias_v", shape=(d,)))
            lib.ea_add_2d(N, d, dqv.data_ptr(), ops.dt(dqv), d, dqkv.data_ptr(), ops.dt(dqkv), 3 * d, 1.0,
                          ops.stream())
        qkv_w = b.w(A + "linear_q.weight", A + "linear_k.weight", A + "linear_v.weight", shape=(3 * d, d))
        # linear_pos: dp[h] = sum_b dBD[h][b]^T qv[b, :, h]  (K = B*T), dWpos = dp^T pos; with the
        # shifted layout the GEMM runs over every physical column and rows [shift, shift + P2) of
        # its output are dp

        def dpp_wgrad(after=None):
            with ops.wgrad(dbd, qv, pos, after=after, launches=True):
                Mp = P2 + shift if shift else P2
                dpp_full = empty(Mp, d, dtype=cd, device=dev)
                ops.gemm(dbd, qv, dpp_full, M=Mp, N=dk, K=B * T, a_kmajor=0, b_kmajor=0, lda=ldbd, ldb=d, ldc=d,
                         batch=1, nh=H, sA=(0, B * T * ldbd), sB=(0, dk), sC=(0, dk))
                ops.linear_dw(dpp_full[shift:], pos, b.g(A + "linear_pos.weight"), accumulate=True)

        fork = ops.fork_event()
        if fork is None:
            dpp_wgrad()
        with ops.wgrad(dqkv, xn2):
            ops.colsum(dqkv, b.g(A + "linear_q.bias", A + "linear_k.bias", A + "linear_v.bias", shape=(3 * d,)))
            ops.linear_dw(dqkv, xn2, b.g(A + "linear_q.weight", A + "linear_k.weight", A + "linear_v.weight",
                                          shape=(3 * d, d)), accumulate=True)
        dxn2 = empty(N, d, dtype=cd, device=dev)
        ops.linear_dx(dqkv, qkv_w, dxn2)
        if fork is not None:  # the side GEMM issued after the main chain's next kernel (fork_event)
            dpp_wgrad(after=fork)
        del dbd
        dv_ff1 = dv_buf(N, d, cd, dev)
        ln_bwd(dxn2, x1, b, "norm_mha", mu2, rs2, dx, accumulate=True,
               drop=drop_arg(dv_ff1, L.ff_scale, p, sd(2), b.g("feed_forward_macaron.w_2.bias")))
        # ---- macaron FFN
        _ffn_bwd(L, b, dx, x0, s_ff1, "feed_forward_macaron", "norm_ff_macaron", p, sd(1), sd(2), dv_in=dv_ff1)
        ops.grad_ready(b)
        return dx.view(B, T, d), None, None, None, None, None
