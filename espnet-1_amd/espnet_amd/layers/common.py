"""Shared plumbing of the block-level autograd Functions.

Each Function's forward launches the block's HIP kernels and keeps its intermediates;
its backward launches the hand-written backward kernels and writes parameter gradients
straight into the gradient arena (the Parameters are views, autograd never sees them).
Only activations flow through autograd, so a whole training step is ~25 autograd nodes.
"""
from __future__ import annotations

import ctypes
import math
import os

import torch

from .. import hip_ops as ops
from .._lib import (ACT_NONE, ACT_RELU, ACT_SWISH, EPI_ACT, EPI_DACT, EPI_RESID, EPI_STORE,
                    lib)

__all__ = ["Bound", "rup", "empty", "ops", "lib", "EPI_ACT", "EPI_DACT", "EPI_RESID",
           "EPI_STORE", "ACT_NONE", "ACT_RELU", "ACT_SWISH", "site_seed", "attn_fwd", "attn_bwd",
           "LayerNormFn", "ln_fwd", "ln_bwd", "math", "F32", "fused_attn_ok", "attn_dmask", "ptr",
           "attn_fused_bwd", "dv_buf", "drop_arg", "site_dv", "multisequential_draw"]

F32 = torch.float32


def rup(n, m=8):
    return (n + m - 1) // m * m


def empty(*shape, dtype=F32, device="cuda"):
    if len(shape) == 1 and isinstance(shape[0], (tuple, list, torch.Size)):
        shape = tuple(shape[0])
    return torch.empty(shape, dtype=dtype, device=device)


FUSED_ATTN = os.environ.get("EA_FUSED_ATTN", "1") != "0"


def fused_attn_ok(cd, dk, T1, T2) -> bool:
    """The fused attention kernels (relattn.hip) take bf16 operands and head dim 64 (any
    lengths); other cases use the unfused path."""
    return FUSED_ATTN and cd == torch.bfloat16 and dk == 64 and T1 >= 1 and T2 >= 1


def ptr(t) -> int:
    return 0 if t is None else t.data_ptr()


def attn_dmask(rows, T2, p, device):
    """Dropout keep-bit buffer of the fused attention (ea_attn_fused_fwd2 writes it, the
    backward reads it instead of rehashing): rows x ldm uint32 words, or (None, 0) when p == 0."""
    if p <= 0:
        return None, 0
    ldm = 2 * ((T2 + 63) // 64)
    return torch.empty(rows * ldm, dtype=torch.int32, device=device), ldm


def dbd_layout(T1: int):
    """(shift, row stride) of the band gradient written by the pipelined dQ pass
    (ea_attn_dbd_layout: logical column r at physical r + shift, 16-B aligned band windows)."""
    sh, ld = ctypes.c_int(0), ctypes.c_long(0)
    rc = lib.ea_attn_dbd_layout(int(T1), ctypes.addressof(sh), ctypes.addressof(ld))
    if rc != 0:
        raise RuntimeError(f"ea_attn_dbd_layout({T1}) failed: {rc}")
    return sh.value, ld.value


def attn_fused_bwd(*, B, H, T1, T2, q, ldq, k, ldk, v, ldv, bu, bv, pp, ldp, klen, causal, scale, p, seed,
                   O, ldo, lse, dO, lddo, dq, lddq, dk, lddk, dv, lddv, dbd=None, ldbd=0, part=None,
                   ldpart=0, qv_out=None, ldqv=0, dmask=None, ldm=0, flags=0):
    """ea_attn_fused_bwd2 with its workspace (D_i, q+u, q+v handed between the two passes),
    a stream-ordered allocation freed behind the launches."""
    n = ctypes.c_long(0)
    lib.ea_attn_fused_bwd_ws_bytes(B, H, T1, ctypes.addressof(n))
    ws = torch.empty(n.value, dtype=torch.uint8, device=dO.device)
    lib.ea_attn_fused_bwd2(B, H, T1, T2, 64, ptr(q), ldq, ptr(k), ldk, ptr(v), ldv, ptr(bu), ptr(bv), ptr(pp),
                           ldp, ptr(klen), int(causal), float(scale), float(p), seed, ptr(O), ldo, ptr(lse),
                           ptr(dO), lddo, ptr(dq), lddq, ptr(dk), lddk, ptr(dv), lddv, ptr(dbd), ldbd, ptr(part),
                           ldpart, ptr(qv_out), ldqv, ptr(dmask), ldm, ws.data_ptr(), n.value, flags, ops.stream())


def multisequential_draw(n: int):
    """MultiSequential.forward (espnet/nets/pytorch_backend/transformer/repeat.py:27) draws
    `torch.empty(len(self)).uniform_()` from torch's default CPU generator on every forward,
    training or not (its layer-drop decisions; rate 0 in the recipes).  The build draws the
    same numbers at the same point so the host RNG stream the reference's SpecAug / TimeWarp
    read next step stays aligned.  A captured step makes its draws before the replay
    (train/graph.py) and suppresses these with SKIP_LAYERDROP_DRAWS."""
    if not SKIP_LAYERDROP_DRAWS:
        torch.empty(n).uniform_()


SKIP_LAYERDROP_DRAWS = False


def site_seed(base: int, layer: int, site: int) -> int:
    """Distinct dropout stream per (step, layer, site); forward and backward share it."""
    z = (base * 0x9E3779B97F4A7C15 + layer * 0xBF58476D1CE4E5B9 + site * 0x94D049BB133111EB)
    return z & 0xFFFFFFFFFFFFFFFF


class Bound:
    """Arena views of one module's parameters: w() in the compute dtype (the bf16 shadow
    under AMP), f() the f32 master, g() the f32 gradient."""

    def __init__(self, arena, prefix: str, cd):
        self.arena = arena
        self.prefix = prefix
        self.cd = cd
        self._cache = {}

    def _v(self, which, names, shape):
        key = (which, names, shape)
        t = self._cache.get(key)
        if t is None:
            t = self.arena.view([self.prefix + n for n in names], shape, which)
            self._cache[key] = t
        return t

    def w(self, *names, shape=None):
        return self._v("shadow" if self.cd != F32 else "data", names, shape)

    def f(self, *names, shape=None):
        return self._v("data", names, shape)

    def g(self, *names, shape=None):
        return self._v("grad", names, shape)


def _n(name, leaf):
    return f"{name}.{leaf}" if name else leaf


def ln_fwd(x2d, b: Bound, name: str, out_dtype):
    N, d = x2d.shape
    y = empty(N, d, dtype=out_dtype, device=x2d.device)
    mu = empty(N, device=x2d.device)
    rs = empty(N, device=x2d.device)
    ops.layernorm_fwd(x2d, b.f(_n(name, "weight")), b.f(_n(name, "bias")), y, mu, rs)
    return y, mu, rs


def ln_bwd(dy, x2d, b: Bound, name: str, mu, rs, dx, accumulate=True, drop=None):
    ops.layernorm_bwd(dy, x2d, b.f(_n(name, "weight")), mu, rs, dx, b.g(_n(name, "weight")),
                      b.g(_n(name, "bias")), accumulate=accumulate, drop=drop)


# Every norm_* backward of a Conformer / Transformer block is followed by a residual dropout
# backward (the next sub-block's output dropout, walking backward): with FUSE_LN_DROP the
# LayerNorm kernel writes that site's dv = dropout(scale * dx) from the dx it has just finished
# (ea_layernorm_bwd_drop), and the site keeps only the bias column sum.
FUSE_LN_DROP = os.environ.get("EA_FUSE_LN_DROP", "1") != "0"


def dv_buf(N, d, cd, dev):
    """Pre-allocated dv of the next site when the LayerNorm backward writes it, else None."""
    return empty(N, d, dtype=cd, device=dev) if FUSE_LN_DROP and cd == torch.bfloat16 else None


def drop_arg(dv, scale, p, seed, bias_g):
    """The LayerNorm backward's drop= argument: write dv and add its column sums to bias_g."""
    return None if dv is None else (dv, scale, p, seed, bias_g)


def site_dv(dx, dv, bias_g, scale, p, seed, cd):
    """dv = dropout(scale * dx) and bias_g += its column sums at a residual site; both already
    done by the preceding LayerNorm backward when dv is given."""
    if dv is not None:
        return dv
    N, d = dx.shape
    dv = empty(N, d, dtype=cd, device=dx.device)
    ops.scale_dropout_colsum(dx, dv, bias_g, scale=scale, p=p, seed=seed)
    return dv


class LayerNormFn(torch.autograd.Function):
    """LayerNorm (eps 1e-12) on the f32 residual stream -> f32 (after_norm)."""

    @staticmethod
    def forward(ctx, x, module):
        shp = x.shape
        x2 = x.reshape(-1, shp[-1])
        y, mu, rs = ln_fwd(x2, module._b, "", F32)
        if torch.is_grad_enabled() or x.requires_grad:
            ctx.save = (x2, mu, rs, module)
        return y.view(shp)

    @staticmethod
    def backward(ctx, dy):
        x2, mu, rs, module = ctx.save
        dy2 = dy.reshape(-1, x2.shape[-1]).contiguous()
        dx = torch.empty_like(x2)
        ln_bwd(dy2, x2, module._b, "", mu, rs, dx, accumulate=False)
        ops.grad_ready(module._b)
        return dx.view(dy.shape), None


# ----------------------------------------------------------------------------- attention core
def attn_fwd(q, k, v, *, B, H, T1, T2, dk, ldq, ldk, ldv, klen, causal, scale, p, seed, cd,
             bd=None, ldbd=0):
    """softmax(scale*(q k^T [+ rel_shift(bd)]) masked) -> dropout -> @ v, all (b,h) at once.
    q/k/v are row views (row strides ldq/ldk/ldv, head h at column h*dk).  Returns
    O (B*T1, H*dk) cd, P (f32 softmax), Pd (dropout(P) in cd), ldT."""
    dev = q.device
    ldT = rup(T2, 8)
    S = empty(B * H * T1 * ldT, device=dev)
    ops.gemm(q, k, S, M=T1, N=T2, K=dk, a_kmajor=1, b_kmajor=1, lda=ldq, ldb=ldk, ldc=ldT,
             batch=B, nh=H, sA=(T1 * ldq, dk), sB=(T2 * ldk, dk), sC=(H * T1 * ldT, T1 * ldT),
             splitk=False)
    Pd = empty(B * H * T1 * ldT, dtype=cd, device=dev)
    lib.ea_attn_softmax_fwd(B, H, T1, T2, scale, S.data_ptr(), ldT,
                            0 if bd is None else bd.data_ptr(), ldbd,
                            0 if klen is None else klen.data_ptr(), int(causal), float(p),
                            seed, S.data_ptr(), ldT, Pd.data_ptr(), ops.dt(Pd), ldT, ops.stream())
    O = empty(B * T1, H * dk, dtype=cd, device=dev)
    ops.gemm(Pd, v, O, M=T1, N=dk, K=T2, a_kmajor=1, b_kmajor=0, lda=ldT, ldb=ldv, ldc=H * dk,
             batch=B, nh=H, sA=(H * T1 * ldT, T1 * ldT), sB=(T2 * ldv, dk), sC=(T1 * H * dk, dk),
             splitk=False)
    return O, S, Pd, ldT


def attn_bwd(dO, q, k, v, P, Pd, ldT, *, B, H, T1, T2, dk, ldq, ldk, ldv, scale, p, seed, cd,
             dq, lddq, dk_, lddk, dv, lddv, dbd=None, ldbd=0):
    """Backward of attn_fwd: writes dq (scaled scores grad . k), dk_, dv; optionally the
    rel-pos band gradient dbd [h][b][i][ldbd]."""
    dev = dO.device
    d = H * dk
    dPd = empty(B * H * T1 * ldT, device=dev)
    ops.gemm(dO, v, dPd, M=T1, N=T2, K=dk, a_kmajor=1, b_kmajor=1, lda=d, ldb=ldv, ldc=ldT,
             batch=B, nh=H, sA=(T1 * d, dk), sB=(T2 * ldv, dk), sC=(H * T1 * ldT, T1 * ldT),
             splitk=False)
    dS = empty(B * H * T1 * ldT, dtype=cd, device=dev)
    lib.ea_attn_softmax_bwd(B, H, T1, T2, scale, dPd.data_ptr(), ldT, P.data_ptr(), ldT, float(p),
                            seed, dS.data_ptr(), ops.dt(dS), ldT,
                            0 if dbd is None else dbd.data_ptr(), ldbd, ops.stream())
    zs = (H * T1 * ldT, T1 * ldT)
    ops.gemm(dS, k, dq, M=T1, N=dk, K=T2, a_kmajor=1, b_kmajor=0, lda=ldT, ldb=ldk, ldc=lddq,
             batch=B, nh=H, sA=zs, sB=(T2 * ldk, dk), sC=(T1 * lddq, dk), splitk=False)
    ops.gemm(dS, q, dk_, M=T2, N=dk, K=T1, a_kmajor=0, b_kmajor=0, lda=ldT, ldb=ldq, ldc=lddk,
             batch=B, nh=H, sA=zs, sB=(T1 * ldq, dk), sC=(T2 * lddk, dk), splitk=False)
    ops.gemm(Pd, dO, dv, M=T2, N=dk, K=T1, a_kmajor=0, b_kmajor=0, lda=ldT, ldb=d, ldc=lddv,
             batch=B, nh=H, sA=zs, sB=(T1 * d, dk), sC=(T2 * lddv, dk), splitk=False)
