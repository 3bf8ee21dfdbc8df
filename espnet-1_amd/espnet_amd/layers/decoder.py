"""TransformerDecoder training forward — espnet2/asr/decoder/transformer_decoder.py:92-145
with DecoderLayer (transformer/decoder_layer.py:63-134, normalize_before=True,
concat_after=False), Embedding + PositionalEncoding (embedding.py:81-92) and the output
Linear — as ONE autograd node (`DecoderFn`).

MI355X layout choice: the encoder memory is projected to the cross-attention keys and
values of ALL decoder layers by a single GEMM (N = 2*d*num_blocks = 6144 columns for C3)
— the six layers' src_attn.linear_k/linear_v weights are adjacent in the parameter arena —
and its backward is likewise one dW GEMM and one dX GEMM with K = 6144.
"""
from __future__ import annotations

import math

import torch
from torch import nn

from .common import (ACT_RELU, EPI_ACT, EPI_DACT, EPI_RESID, EPI_STORE, F32, Bound, attn_bwd,
                     attn_dmask, attn_fused_bwd, attn_fwd, empty, fused_attn_ok, lib, ln_bwd, ln_fwd, ops, ptr,
                     site_seed, dv_buf, drop_arg, site_dv)


def _mha_fwd(q, k, v, *, B, H, T1, T2, dk, ldq, ldk, ldv, klen, causal, scale, p, seed, cd):
    """Scaled dot-product core of MultiHeadedAttention (attention.py:63-93) with the key
    padding (+ causal) mask: the fused flash kernel (relattn.hip, no positional term) when
    eligible, else the unfused GEMM + softmax path.  Returns (O, saved state)."""
    if fused_attn_ok(cd, dk, T1, T2):
        O = empty(B * T1, H * dk, dtype=cd, device=q.device)
        lse = empty(B * H * T1, device=q.device)
        dmask, ldm = attn_dmask(B * H * T1, T2, p, q.device)
        lib.ea_attn_fused_fwd2(B, H, T1, T2, dk, q.data_ptr(), ldq, k.data_ptr(), ldk, v.data_ptr(), ldv,
                               None, None, None, 0, klen.data_ptr(), int(causal), scale, float(p), seed,
                               O.data_ptr(), H * dk, lse.data_ptr(), ptr(dmask), ldm, ops.stream())
        return O, ("fused", O, lse, dmask, ldm)
    O, P, Pd, ldT = attn_fwd(q, k, v, B=B, H=H, T1=T1, T2=T2, dk=dk, ldq=ldq, ldk=ldk, ldv=ldv, klen=klen,
                             causal=causal, scale=scale, p=p, seed=seed, cd=cd)
    return O, ("unfused", P, Pd, ldT)


def _mha_bwd(st, dO, q, k, v, *, B, H, T1, T2, dk, ldq, ldk, ldv, klen, causal, scale, p, seed, cd,
             dq, lddq, dk_, lddk, dv, lddv):
    if st[0] == "fused":
        _, O, lse, dmask, ldm = st
        attn_fused_bwd(B=B, H=H, T1=T1, T2=T2, q=q, ldq=ldq, k=k, ldk=ldk, v=v, ldv=ldv, bu=None, bv=None, pp=None,
                       ldp=0, klen=klen, causal=causal, scale=scale, p=p, seed=seed, O=O, ldo=H * dk, lse=lse,
                       dO=dO, lddo=H * dk, dq=dq, lddq=lddq, dk=dk_, lddk=lddk, dv=dv, lddv=lddv, dmask=dmask,
                       ldm=ldm)
        return
    _, P, Pd, ldT = st
    attn_bwd(dO, q, k, v, P, Pd, ldT, B=B, H=H, T1=T1, T2=T2, dk=dk, ldq=ldq, ldk=ldk, ldv=ldv, scale=scale,
             p=p, seed=seed, cd=cd, dq=dq, lddq=lddq, dk_=dk_, lddk=lddk, dv=dv, lddv=lddv)
from .conformer import LayerNorm, MultiHeadedAttention, PositionwiseFeedForward


def sinusoid_table(n, d):
    """PositionalEncoding.extend_pe (embedding.py:60-79), a construction-time constant."""
    pe = torch.zeros(n, d)
    pos = torch.arange(0, n, dtype=torch.float32).unsqueeze(1)
    div = torch.exp(torch.arange(0, d, 2, dtype=torch.float32) * -(math.log(10000.0) / d))
    pe[:, 0::2] = torch.sin(pos * div)
    pe[:, 1::2] = torch.cos(pos * div)
    return pe


class PositionalEncoding(nn.Module):
    """embedding.py:35-92: x * sqrt(d) + pe[t], dropout (the table is a constant, not in
    the state_dict)."""

    absolute = True

    def __init__(self, d_model, dropout_rate, max_len=5000):
        super().__init__()
        self.d_model = d_model
        self.xscale = math.sqrt(d_model)
        self.dropout_rate = dropout_rate
        self.max_len = max_len
        self._pe = None

    def table(self, L, device):
        if self._pe is None or self._pe.shape[0] < L or self._pe.device != device:
            self._pe = sinusoid_table(max(self.max_len, L), self.d_model).to(device)
        return self._pe


class DecoderLayer(nn.Module):
    """transformer/decoder_layer.py:22-61 parameter set."""

    def __init__(self, size, self_attn, src_attn, feed_forward, dropout_rate,
                 normalize_before=True, concat_after=False):
        super().__init__()
        if not normalize_before or concat_after:
            raise NotImplementedError("only normalize_before=True, concat_after=False")
        self.size = size
        self.self_attn = self_attn
        self.src_attn = src_attn
        self.feed_forward = feed_forward
        self.norm1 = LayerNorm(size)
        self.norm2 = LayerNorm(size)
        self.norm3 = LayerNorm(size)
        self.dropout_rate = dropout_rate


def decoder_arena_groups(prefix, num_blocks):
    g = []
    for i in range(num_blocks):
        a = f"{prefix}decoders.{i}.self_attn."
        g.append([a + "linear_q.weight", a + "linear_k.weight", a + "linear_v.weight"])
        g.append([a + "linear_q.bias", a + "linear_k.bias", a + "linear_v.bias"])
    kw, kb = [], []
    for i in range(num_blocks):
        a = f"{prefix}decoders.{i}.src_attn."
        kw += [a + "linear_k.weight", a + "linear_v.weight"]
        kb += [a + "linear_k.bias", a + "linear_v.bias"]
    return g + [kw, kb]


def _kv_names(nb):
    w, b = [], []
    for i in range(nb):
        a = f"decoders.{i}.src_attn."
        w += [a + "linear_k.weight", a + "linear_v.weight"]
        b += [a + "linear_k.bias", a + "linear_v.bias"]
    return w, b


class DecoderFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, memory, hlens, ys_in, ys_in_lens, dec, seed, training):
        b = dec._b
        cd = b.cd
        B, Tm, d = memory.shape
        L = ys_in.shape[1]
        N, Nm = B * L, B * Tm
        nb = len(dec.decoders)
        H = dec.decoders[0].self_attn.h
        dk = d // H
        V = dec.output_layer.out_features
        dev = memory.device
        p = dec.dropout_rate if training else 0.0
        p_sa = dec.self_attention_dropout_rate if training else 0.0
        p_src = dec.src_attention_dropout_rate if training else 0.0
        p_pos = dec.embed[1].dropout_rate if training else 0.0
        sd = lambda l, s: site_seed(seed, 100 + l, s)  # noqa: E731
        scale = 1.0 / math.sqrt(dk)
        mem = ops.cast(memory.reshape(Nm, d), cd)
        kvw, kvb = _kv_names(nb)
        kv = empty(Nm, 2 * d * nb, dtype=cd, device=dev)
        ops.linear(mem, b.w(*kvw, shape=(2 * d * nb, d)), kv,
                   epi=ops.make_epi(bias=b.f(*kvb, shape=(2 * d * nb,))))
        pe = dec.embed[1]
        x = empty(N, d, device=dev)
        lib.ea_embed_fwd(N, d, L, ys_in.data_ptr(), b.f("embed.0.weight").data_ptr(), pe.xscale,
                         pe.table(L, dev).data_ptr(), p_pos, sd(0, 0), x.data_ptr(), ops.stream())
        saved = []
        ldkv = 2 * d * nb
        for l in range(nb):
            n = f"decoders.{l}."
            sa, xa = n + "self_attn.", n + "src_attn."
            # self-attention (causal & target padding mask, transformer_decoder.py:117-122)
            xn1, mu1, rs1 = ln_fwd(x, b, n + "norm1", cd)
            qkv = empty(N, 3 * d, dtype=cd, device=dev)
            ops.linear(xn1, b.w(sa + "linear_q.weight", sa + "linear_k.weight", sa + "linear_v.weight",
                                shape=(3 * d, d)), qkv,
                       epi=ops.make_epi(bias=b.f(sa + "linear_q.bias", sa + "linear_k.bias",
                                                 sa + "linear_v.bias", shape=(3 * d,))))
            O1, st1 = _mha_fwd(qkv, qkv[:, d:], qkv[:, 2 * d:], B=B, H=H, T1=L, T2=L, dk=dk,
                               ldq=3 * d, ldk=3 * d, ldv=3 * d, klen=ys_in_lens, causal=True,
                               scale=scale, p=p_sa, seed=sd(l, 1), cd=cd)
            x1 = empty(N, d, device=dev)
            ops.linear(O1, b.w(sa + "linear_out.weight"), x1,
                       epi=ops.make_epi(EPI_RESID, bias=b.f(sa + "linear_out.bias"), resid=x,
                                        drop_p=p, seed=sd(l, 2)))
            # source attention over the encoder memory (memory_mask, :125-127)
            xn2, mu2, rs2 = ln_fwd(x1, b, n + "norm2", cd)
            q2 = empty(N, d, dtype=cd, device=dev)
            ops.linear(xn2, b.w(xa + "linear_q.weight"), q2, epi=ops.make_epi(bias=b.f(xa + "linear_q.bias")))
            k2 = kv[:, 2 * d * l:]
            v2 = kv[:, 2 * d * l + d:]
            O2, st2 = _mha_fwd(q2, k2, v2, B=B, H=H, T1=L, T2=Tm, dk=dk, ldq=d, ldk=ldkv,
                               ldv=ldkv, klen=hlens, causal=False, scale=scale, p=p_src,
                               seed=sd(l, 3), cd=cd)
            x2 = empty(N, d, device=dev)
            ops.linear(O2, b.w(xa + "linear_out.weight"), x2,
                       epi=ops.make_epi(EPI_RESID, bias=b.f(xa + "linear_out.bias"), resid=x1,
                                        drop_p=p, seed=sd(l, 4)))
            # feed-forward (ReLU)
            xn3, mu3, rs3 = ln_fwd(x2, b, n + "norm3", cd)
            Fh = dec.decoders[l].feed_forward.w_1.out_features
            h = empty(N, Fh, dtype=cd, device=dev)
            a = empty(N, Fh, dtype=cd, device=dev)
            ff = n + "feed_forward."
            ops.linear(xn3, b.w(ff + "w_1.weight"), a,
                       epi=ops.make_epi(EPI_ACT, bias=b.f(ff + "w_1.bias"), act=ACT_RELU, aux=h,
                                        drop_p=p, seed=sd(l, 5)))
            x3 = empty(N, d, device=dev)
            ops.linear(a, b.w(ff + "w_2.weight"), x3,
                       epi=ops.make_epi(EPI_RESID, bias=b.f(ff + "w_2.bias"), resid=x2,
                                        drop_p=p, seed=sd(l, 6)))
            saved.append((x, x1, x2, (xn1, mu1, rs1, qkv, O1, st1),
                          (xn2, mu2, rs2, q2, O2, st2), (xn3, mu3, rs3, h, a)))
            x = x3
        xf, muf, rsf = ln_fwd(x, b, "after_norm", cd)
        logits = empty(N, V, device=dev)
        ops.linear(xf, b.w("output_layer.weight"), logits,
                   epi=ops.make_epi(bias=b.f("output_layer.bias")))
        ctx.dec = dec
        ctx.meta = (B, Tm, L, d, H, dk, nb, p, p_sa, p_src, p_pos, seed, scale)
        ctx.save = (mem, kv, ys_in, saved, x, xf, muf, rsf, hlens, ys_in_lens)
        return logits.view(B, L, V)

    @staticmethod
    def backward(ctx, dlogits):
        dec = ctx.dec
        b = dec._b
        cd = b.cd
        B, Tm, L, d, H, dk, nb, p, p_sa, p_src, p_pos, seed, scale = ctx.meta
        mem, kv, ys_in, saved, xlast, xf, muf, rsf, hlens, ys_in_lens = ctx.save
        ctx.save = None
        sd = lambda l, s: site_seed(seed, 100 + l, s)  # noqa: E731
        N, Nm = B * L, B * Tm
        V = dlogits.shape[-1]
        dev = dlogits.device
        dlog = ops.cast(dlogits.reshape(N, V).contiguous(), cd)
        with ops.wgrad(dlog, xf):
            ops.colsum(dlog, b.g("output_layer.bias"))
            ops.linear_dw(dlog, xf, b.g("output_layer.weight"), accumulate=True)
        dxf = empty(N, d, dtype=cd, device=dev)
        ops.linear_dx(dlog, b.w("output_layer.weight"), dxf)
        dx = empty(N, d, device=dev)
        # each norm backward also writes the dropout backward of the site below it (dv_buf)
        dv_ff = dv_buf(N, d, cd, dev) if nb > 0 else None
        ln_bwd(dxf, xlast, b, "after_norm", muf, rsf, dx, accumulate=False,
               drop=None if dv_ff is None else
               drop_arg(dv_ff, 1.0, p, sd(nb - 1, 6), b.g(f"decoders.{nb - 1}.feed_forward.w_2.bias")))
        ldkv = 2 * d * nb
        dkv = empty(Nm, ldkv, dtype=cd, device=dev)
        for l in reversed(range(nb)):
            n = f"decoders.{l}."
            sa, xa, ff = n + "self_attn.", n + "src_attn.", n + "feed_forward."
            x0, x1, x2, s1, s2, s3 = saved[l]
            # feed-forward
            xn3, mu3, rs3, h, a = s3
            dv = site_dv(dx, dv_ff, b.g(ff + "w_2.bias"), 1.0, p, sd(l, 6), cd)
            with ops.wgrad(dv, a):
                ops.linear_dw(dv, a, b.g(ff + "w_2.weight"), accumulate=True)
            # the layer above's weight gradients on the side stream (beside this layer's latency-
            # bound backward instead of in the end-of-pass grouped GEMM), forked here and issued
            # after this layer's first GEMM (which keeps the main chain's queue)
            fork = ops.fork_event() if l < nb - 1 else None
            dh = empty(*h.shape, dtype=cd, device=dev)
            ops.linear_dx(dv, b.w(ff + "w_2.weight"), dh,
                          epi=ops.make_epi(EPI_DACT, act=ACT_RELU, aux=h, drop_p=p, seed=sd(l, 5)))
            if fork is not None:
                ops.flush_wgrad_side(after=fork)
            with ops.wgrad(dh, xn3):
                ops.colsum(dh, b.g(ff + "w_1.bias"))
                ops.linear_dw(dh, xn3, b.g(ff + "w_1.weight"), accumulate=True)
            dxn = empty(N, d, dtype=cd, device=dev)
            ops.linear_dx(dh, b.w(ff + "w_1.weight"), dxn)
            dv_src = dv_buf(N, d, cd, dev)
            ln_bwd(dxn, x2, b, n + "norm3", mu3, rs3, dx, accumulate=True,
                   drop=drop_arg(dv_src, 1.0, p, sd(l, 4), b.g(xa + "linear_out.bias")))
            # source attention
            xn2, mu2, rs2, q2, O2, st2 = s2
            dv = site_dv(dx, dv_src, b.g(xa + "linear_out.bias"), 1.0, p, sd(l, 4), cd)
            with ops.wgrad(dv, O2):
                ops.linear_dw(dv, O2, b.g(xa + "linear_out.weight"), accumulate=True)
            dO = empty(N, d, dtype=cd, device=dev)
            ops.linear_dx(dv, b.w(xa + "linear_out.weight"), dO)
            dq = empty(N, d, dtype=cd, device=dev)
            _mha_bwd(st2, dO, q2, kv[:, 2 * d * l:], kv[:, 2 * d * l + d:], B=B, H=H, T1=L, T2=Tm, dk=dk,
                     ldq=d, ldk=ldkv, ldv=ldkv, klen=hlens, causal=False, scale=scale, p=p_src,
                     seed=sd(l, 3), cd=cd, dq=dq, lddq=d, dk_=dkv[:, 2 * d * l:], lddk=ldkv,
                     dv=dkv[:, 2 * d * l + d:], lddv=ldkv)
            with ops.wgrad(dq, xn2):
                ops.colsum(dq, b.g(xa + "linear_q.bias"))
                ops.linear_dw(dq, xn2, b.g(xa + "linear_q.weight"), accumulate=True)
            dxn = empty(N, d, dtype=cd, device=dev)
            ops.linear_dx(dq, b.w(xa + "linear_q.weight"), dxn)
            dv_self = dv_buf(N, d, cd, dev)
            ln_bwd(dxn, x1, b, n + "norm2", mu2, rs2, dx, accumulate=True,
                   drop=drop_arg(dv_self, 1.0, p, sd(l, 2), b.g(sa + "linear_out.bias")))
            # self attention
            xn1, mu1, rs1, qkv, O1, st1 = s1
            dv = site_dv(dx, dv_self, b.g(sa + "linear_out.bias"), 1.0, p, sd(l, 2), cd)
            with ops.wgrad(dv, O1):
                ops.linear_dw(dv, O1, b.g(sa + "linear_out.weight"), accumulate=True)
            dO = empty(N, d, dtype=cd, device=dev)
            ops.linear_dx(dv, b.w(sa + "linear_out.weight"), dO)
            dqkv = empty(N, 3 * d, dtype=cd, device=dev)
            _mha_bwd(st1, dO, qkv, qkv[:, d:], qkv[:, 2 * d:], B=B, H=H, T1=L, T2=L, dk=dk,
                     ldq=3 * d, ldk=3 * d, ldv=3 * d, klen=ys_in_lens, causal=True, scale=scale, p=p_sa,
                     seed=sd(l, 1), cd=cd, dq=dqkv, lddq=3 * d, dk_=dqkv[:, d:], lddk=3 * d,
                     dv=dqkv[:, 2 * d:], lddv=3 * d)
            wn = (sa + "linear_q.weight", sa + "linear_k.weight", sa + "linear_v.weight")
            bn = (sa + "linear_q.bias", sa + "linear_k.bias", sa + "linear_v.bias")
            with ops.wgrad(dqkv, xn1):
                ops.colsum(dqkv, b.g(*bn, shape=(3 * d,)))
                ops.linear_dw(dqkv, xn1, b.g(*wn, shape=(3 * d, d)), accumulate=True)
            dxn = empty(N, d, dtype=cd, device=dev)
            ops.linear_dx(dqkv, b.w(*wn, shape=(3 * d, d)), dxn)
            dv_ff = dv_buf(N, d, cd, dev) if l > 0 else None  # layer l-1's feed-forward site
            ln_bwd(dxn, x0, b, n + "norm1", mu1, rs1, dx, accumulate=True,
                   drop=None if dv_ff is None else
                   drop_arg(dv_ff, 1.0, p, sd(l - 1, 6), b.g(f"decoders.{l - 1}.feed_forward.w_2.bias")))
        pe = dec.embed[1]
        lib.ea_embed_bwd(N, d, ys_in.data_ptr(), dx.data_ptr(), pe.xscale, p_pos, sd(0, 0),
                         b.g("embed.0.weight").data_ptr(), ops.stream())
        kvw, kvb = _kv_names(nb)
        with ops.wgrad(dkv, mem):
            ops.colsum(dkv, b.g(*kvb, shape=(ldkv,)))
            ops.linear_dw(dkv, mem, b.g(*kvw, shape=(ldkv, d)), accumulate=True)
        dmem = empty(Nm, d, device=dev)
        ops.linear_dx(dkv, b.w(*kvw, shape=(ldkv, d)), dmem)
        ops.grad_ready(b)
        return dmem.view(B, Tm, d), None, None, None, None, None, None
