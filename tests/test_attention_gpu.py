"""Fused attention kernels (relattn.hip: ea_attn_fused_fwd(2) / ea_attn_fused_bwd2) against an fp32
PyTorch restatement of RelPositionMultiHeadedAttention / MultiHeadedAttention
(espnet/nets/pytorch_backend/transformer/attention.py:15-111, 209-305; rel_shift :237-260)
on the same bf16-rounded inputs, and against the unfused HIP path (same dropout masks)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
bf = torch.bfloat16


def rel_shift(x):
    """attention.py:237-260 (zero_triu=False)."""
    zero_pad = torch.zeros((*x.size()[:3], 1), device=x.device, dtype=x.dtype)
    x_padded = torch.cat([zero_pad, x], dim=-1)
    x_padded = x_padded.view(*x.size()[:2], x.size(3) + 1, x.size(2))
    return x_padded[:, :, 1:].view_as(x)[:, :, :, : x.size(-1) // 2 + 1]


def reference(q, k, v, u, vb, pp, klen, causal, H):
    """fp32 torch: q (B,T1,H*64), k/v (B,T2,H*64), pp (2T-1, H*64) or None."""
    B, T1, d = q.shape
    T2 = k.shape[1]
    dk = d // H
    qh = q.view(B, T1, H, dk).transpose(1, 2)
    kh = k.view(B, T2, H, dk).transpose(1, 2)
    vh = v.view(B, T2, H, dk).transpose(1, 2)
    if pp is not None:
        ac = torch.matmul(qh + u.view(1, H, 1, dk), kh.transpose(-2, -1))
        ph = pp.view(1, -1, H, dk).transpose(1, 2)
        bd = rel_shift(torch.matmul(qh + vb.view(1, H, 1, dk), ph.transpose(-2, -1)))
        scores = (ac + bd) / math.sqrt(dk)
    else:
        scores = torch.matmul(qh, kh.transpose(-2, -1)) / math.sqrt(dk)
    mask = torch.arange(T2, device=q.device)[None, :] < klen[:, None]  # (B, T2)
    mask = mask[:, None, None, :].expand(B, 1, T1, T2)
    if causal:
        mask = mask & torch.tril(torch.ones(T1, T2, dtype=torch.bool, device=q.device))[None, None]
    scores = scores.masked_fill(~mask, torch.finfo(scores.dtype).min)
    attn = torch.softmax(scores, dim=-1).masked_fill(~mask, 0.0)
    x = torch.matmul(attn, vh)
    return x.transpose(1, 2).reshape(B, T1, d)


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


def dbd_layout(T1, v2):
    """(shift, row stride) of the band gradient: v2 = the pipelined dQ pass's shifted layout
    (ea_attn_dbd_layout), else logical columns at 0."""
    import ctypes
    from espnet_amd._lib import lib
    if not v2:
        return 0, (2 * T1 - 1 + 7) // 8 * 8
    sh, ld = ctypes.c_int(0), ctypes.c_long(0)
    assert lib.ea_attn_dbd_layout(T1, ctypes.addressof(sh), ctypes.addressof(ld)) == 0
    assert sh.value >= 15 and (T1 + sh.value) % 8 == 0 and ld.value % 8 == 0
    return sh.value, ld.value


def band_view(dbd, H, B, T1, v2):
    """dbd as (H, B, T1, 2*T1-1) logical columns, plus the physical columns outside them."""
    sh, ld = dbd_layout(T1, v2)
    full = dbd.view(H, B, T1, ld)
    outside = torch.cat([full[..., :sh], full[..., sh + 2 * T1 - 1:]], dim=-1)
    return full[..., sh: sh + 2 * T1 - 1], outside


def run_fused(q, k, v, u, vb, pp, klen, causal, H, dO, p=0.0, seed=0, v2=False):
    """Forward + backward through the C ABI; v2 = the pipelined dQ pass (flags bit 1, shifted
    dbd), else the original pass (flags bit 2)."""
    from espnet_amd import hip_ops as ops
    from espnet_amd._lib import lib
    from espnet_amd.layers.common import attn_fused_bwd
    B, T1, d = q.shape
    T2 = k.shape[1]
    dk = d // H
    O = torch.empty(B, T1, d, dtype=bf, device=DEV)
    lse = torch.empty(B * H * T1, device=DEV)
    ptr = lambda t: 0 if t is None else t.data_ptr()  # noqa: E731
    scale = 1.0 / math.sqrt(dk)
    lib.ea_attn_fused_fwd(B, H, T1, T2, dk, q.data_ptr(), d, k.data_ptr(), d, v.data_ptr(), d, ptr(u), ptr(vb),
                          ptr(pp), d, klen.data_ptr(), int(causal), scale, p, seed, O.data_ptr(), d,
                          lse.data_ptr(), ops.stream())
    dq = torch.empty_like(q)
    dkk = torch.empty_like(k)
    dv = torch.empty_like(v)
    _, ldbd = dbd_layout(T1, v2)
    # NaN-filled: the kernel writes every band row in full (zeros off the band)
    dbd = torch.full((H * B * T1 * ldbd,), float("nan"), dtype=bf, device=DEV) if pp is not None else None
    # the hash path (no keep-bit mask), dq without the rel-pos term (flag bit 0 clear)
    attn_fused_bwd(B=B, H=H, T1=T1, T2=T2, q=q, ldq=d, k=k, ldk=d, v=v, ldv=d, bu=u, bv=vb, pp=pp, ldp=d, klen=klen,
                   causal=causal, scale=scale, p=p, seed=seed, O=O, ldo=d, lse=lse, dO=dO, lddo=d, dq=dq, lddq=d,
                   dk=dkk, lddk=d, dv=dv, lddv=d, dbd=dbd, ldbd=ldbd, flags=2 if v2 else 4)
    torch.cuda.synchronize()
    return O, dq, dkk, dv, dbd, ldbd


def _inputs(B, H, T1, T2, rel, seed=0):
    g = torch.Generator().manual_seed(seed)
    d = H * 64
    r = lambda *s: (torch.randn(*s, generator=g) * 0.5).to(bf).to(DEV)  # noqa: E731
    q, k, v = r(B, T1, d), r(B, T2, d), r(B, T2, d)
    u = (torch.randn(H * 64, generator=g) * 0.1).to(DEV) if rel else None
    vb = (torch.randn(H * 64, generator=g) * 0.1).to(DEV) if rel else None
    pp = r(2 * T1 - 1, d) if rel else None
    dO = r(B, T1, d)
    return q, k, v, u, vb, pp, dO


@pytest.mark.parametrize("v2", [False, True])
@pytest.mark.parametrize("B,H,T1,T2,rel,causal,klens", [
    (2, 3, 137, 137, True, False, [137, 100]),
    (3, 2, 249, 249, True, False, [249, 200, 64]),
    (2, 2, 41, 41, False, True, [41, 30]),
    (2, 2, 41, 137, False, False, [137, 77]),
    (1, 1, 5, 5, True, False, [5]),
    (1, 2, 300, 300, True, False, [300]),
    (2, 1, 41, 300, False, False, [300, 131]),
    (1, 2, 270, 270, False, True, [270]),
    (2, 1, 64, 64, True, False, [64, 1]),
    (1, 1, 130, 130, True, False, [130]),
    # C5's longest bucket: T' = 499 (997-row positional band through the band rings, the
    # T-dependent dbd layout), ragged; decoder self / source attention over 499 frames
    (2, 2, 499, 499, True, False, [499, 331]),
    (1, 1, 499, 499, False, True, [499]),
    (2, 2, 81, 499, False, False, [499, 330]),
])
def test_fused_attention_matches_fp32_reference(B, H, T1, T2, rel, causal, klens, v2):
    q, k, v, u, vb, pp, dO = _inputs(B, H, T1, T2, rel)
    klen = torch.tensor(klens, dtype=torch.long, device=DEV)
    O, dq, dk, dv, dbd, ldbd = run_fused(q, k, v, u, vb, pp, klen, causal, H, dO, v2=v2)
    # fp32 reference on the same (bf16-rounded) inputs; q+u / q+v rounded to bf16 like the kernel
    qf, kf, vf = (t.float().requires_grad_(True) for t in (q, k, v))
    ppf = pp.float().requires_grad_(True) if rel else None
    ref = reference(qf, kf, vf, u, vb, ppf, klen, causal, H)
    valid_q = torch.ones(B, T1, dtype=torch.bool, device=DEV)
    assert _rel(O.float()[valid_q], ref.detach()[valid_q]) < 1e-2
    ref.backward(dO.float())
    assert _rel(dk, kf.grad) < 2e-2
    assert _rel(dv, vf.grad) < 2e-2
    if not rel:
        assert _rel(dq, qf.grad) < 2e-2
        return
    # rel-pos: dq from the kernel is the (q+u) path; the (q+v) path leaves through dbd:
    # dq_total = dq + dBD . pp_h, d pp_h = dBD^T . (q+v)
    d = H * 64
    dbd4, off_band = band_view(dbd, H, B, T1, v2)
    dbd4 = dbd4.float()
    assert off_band.numel() == 0 or float(off_band.float().abs().max()) == 0.0  # zeros, no NaN left
    pph = pp.float().view(2 * T1 - 1, H, 64).permute(1, 0, 2)  # (H, R, 64)
    dq_v = torch.einsum("hbir,hrc->bihc", dbd4, pph).reshape(B, T1, d)
    assert _rel(dq.float() + dq_v, qf.grad) < 2e-2
    qv = (q.float().view(B, T1, H, 64) + vb.view(1, 1, H, 64)).to(bf).float()
    dpp = torch.einsum("hbir,bihc->rhc", dbd4, qv).reshape(2 * T1 - 1, d)
    assert _rel(dpp, ppf.grad) < 2e-2
    # the band structure: dBD[i, r] is zero outside r in [T-1-i, 2T-2-i]
    i = torch.arange(T1, device=DEV)[:, None]
    rr = torch.arange(2 * T1 - 1, device=DEV)[None, :]
    outside = (rr < T1 - 1 - i) | (rr > 2 * T1 - 2 - i)
    assert float(dbd4[:, :, outside].abs().max()) == 0.0


def test_fused_matches_unfused_with_dropout():
    """Same dropout masks (counter hash, index (z*T1 + i)*T2 + j): fused == unfused path."""
    from espnet_amd import hip_ops as ops
    from espnet_amd._lib import lib
    from espnet_amd.layers.common import attn_bwd, attn_fwd
    B, H, T = 2, 2, 97
    q, k, v, u, vb, pp, dO = _inputs(B, H, T, T, True, seed=3)
    klen = torch.tensor([97, 60], dtype=torch.long, device=DEV)
    p, seed = 0.1, 12345
    O, dq, dk, dv, dbd, ldbd = run_fused(q, k, v, u, vb, pp, klen, False, H, dO, p=p, seed=seed)
    d = H * 64
    N = B * T
    P2 = 2 * T - 1
    qu = torch.empty(N, d, dtype=bf, device=DEV)
    qv = torch.empty(N, d, dtype=bf, device=DEV)
    lib.ea_add_pos_bias(N, H, 64, q.data_ptr(), d, u.data_ptr(), vb.data_ptr(), qu.data_ptr(), qv.data_ptr(),
                        ops.dt(qu), ops.stream())
    bd = torch.empty(H * B * T * ldbd, device=DEV)
    ops.gemm(qv, pp, bd, M=T, N=P2, K=64, a_kmajor=1, b_kmajor=1, lda=d, ldb=d, ldc=ldbd, batch=B, nh=H,
             sA=(T * d, 64), sB=(0, 64), sC=(T * ldbd, B * T * ldbd), splitk=False)
    O2, P, Pd, ldT = attn_fwd(qu, k.view(N, d), v.view(N, d), B=B, H=H, T1=T, T2=T, dk=64, ldq=d, ldk=d, ldv=d,
                              klen=klen, causal=False, scale=1 / 8, p=p, seed=seed, cd=bf, bd=bd, ldbd=ldbd)
    dq2 = torch.empty(N, d, dtype=bf, device=DEV)
    dk2 = torch.empty(N, d, dtype=bf, device=DEV)
    dv2 = torch.empty(N, d, dtype=bf, device=DEV)
    dbd2 = torch.empty(H * B * T * ldbd, dtype=bf, device=DEV)
    attn_bwd(dO.view(N, d), qu, k.view(N, d), v.view(N, d), P, Pd, ldT, B=B, H=H, T1=T, T2=T, dk=64, ldq=d, ldk=d,
             ldv=d, scale=1 / 8, p=p, seed=seed, cd=bf, dq=dq2, lddq=d, dk_=dk2, lddk=d, dv=dv2, lddv=d,
             dbd=dbd2, ldbd=ldbd)
    torch.cuda.synchronize()
    assert _rel(O.view(N, d), O2) < 1e-2
    assert _rel(dq.view(N, d), dq2) < 2e-2
    assert _rel(dk.view(N, d), dk2) < 2e-2
    assert _rel(dv.view(N, d), dv2) < 2e-2
    band = dbd2.view(H, B, T, ldbd)[..., :P2]
    assert _rel(dbd.view(H, B, T, ldbd)[..., :P2], band) < 2e-2


@pytest.mark.parametrize("B,H,T,klens,p", [
    (2, 3, 137, [137, 100], 0.0),
    (3, 2, 249, [249, 200, 64], 0.0),
    (1, 2, 300, [300], 0.0),
    (2, 2, 97, [97, 60], 0.1),
    (2, 2, 499, [499, 331], 0.1),
])
def test_fused_bwd2_rel_terms(B, H, T, klens, p):
    """ea_attn_fused_bwd2 with flags=1 and the forward's keep bits: dq includes the (q+v)
    path, per-block column sums give the pos_bias_u / pos_bias_v gradients, qv_out =
    bf16(q + v); dk, dv, dbd equal the flags=0 / rehashing call's bit for bit."""
    from espnet_amd import hip_ops as ops
    from espnet_amd._lib import lib
    from espnet_amd.layers.common import attn_fused_bwd
    q, k, v, u, vb, pp, dO = _inputs(B, H, T, T, True, seed=5)
    klen = torch.tensor(klens, dtype=torch.long, device=DEV)
    seed = 99
    O, dq1, dk1, dv1, dbd1, ldbd = run_fused(q, k, v, u, vb, pp, klen, False, H, dO, p=p, seed=seed)
    d = H * 64
    lse = torch.empty(B * H * T, device=DEV)
    O2 = torch.empty_like(O)
    scale = 1 / 8
    # forward with the dropout keep-bit mask; the backward reads it (bit-identical to rehashing)
    ldm = 2 * ((T + 63) // 64)
    dmask = torch.empty(B * H * T * ldm, dtype=torch.int32, device=DEV) if p > 0 else None
    dmp = 0 if dmask is None else dmask.data_ptr()
    lib.ea_attn_fused_fwd2(B, H, T, T, 64, q.data_ptr(), d, k.data_ptr(), d, v.data_ptr(), d, u.data_ptr(),
                           vb.data_ptr(), pp.data_ptr(), d, klen.data_ptr(), 0, scale, p, seed, O2.data_ptr(), d,
                           lse.data_ptr(), dmp, ldm, ops.stream())
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    dbd = torch.full((H * B * T * ldbd,), float("nan"), dtype=bf, device=DEV)
    nqb = (T + 63) // 64
    part = torch.full((2, B * nqb, d), float("nan"), device=DEV)
    qv = torch.empty(B, T, d, dtype=bf, device=DEV)
    attn_fused_bwd(B=B, H=H, T1=T, T2=T, q=q, ldq=d, k=k, ldk=d, v=v, ldv=d, bu=u, bv=vb, pp=pp, ldp=d, klen=klen,
                   causal=False, scale=scale, p=p, seed=seed, O=O2, ldo=d, lse=lse, dO=dO, lddo=d, dq=dq, lddq=d,
                   dk=dk, lddk=d, dv=dv, lddv=d, dbd=dbd, ldbd=ldbd, part=part, ldpart=d, qv_out=qv, ldqv=d,
                   dmask=dmask, ldm=ldm, flags=1)
    torch.cuda.synchronize()
    assert torch.equal(O2, O) and torch.equal(dk, dk1) and torch.equal(dv, dv1) and torch.equal(dbd, dbd1)
    assert torch.equal(qv, (q.float() + vb.view(1, 1, d)).to(bf))
    # (q+v) path: dq - dq_u = dBD . pp_h on the same bf16 band
    dbd4 = dbd.view(H, B, T, ldbd)[..., : 2 * T - 1].float()
    pph = pp.float().view(2 * T - 1, H, 64).permute(1, 0, 2)
    dq_v = torch.einsum("hbir,hrc->bihc", dbd4, pph).reshape(B, T, d)
    assert _rel(dq.float(), dq1.float() + dq_v) < 1e-2
    # bias partials: sums over each 64-query block of the two dq terms
    du = part[0].sum(0)
    dvb = part[1].sum(0)
    assert _rel(du, dq1.float().sum((0, 1))) < 1e-2
    assert _rel(dvb, dq_v.sum((0, 1))) < 1e-2
    if p == 0.0:  # against the fp32 autograd reference
        qf, kf, vf = (t.float().requires_grad_(True) for t in (q, k, v))
        uf, vbf = u.clone().requires_grad_(True), vb.clone().requires_grad_(True)
        ref = reference(qf, kf, vf, uf, vbf, pp.float(), klen, False, H)
        ref.backward(dO.float())
        assert _rel(dq, qf.grad) < 2e-2
        assert _rel(du, uf.grad) < 2e-2
        assert _rel(dvb, vbf.grad) < 2e-2


@pytest.mark.parametrize("causal,T1,T2,klens", [(True, 45, 45, [45, 30]), (False, 45, 300, [300, 140])])
def test_fused_dropout_mask_matches_rehash(causal, T1, T2, klens):
    """Decoder shapes with dropout: ea_attn_fused_fwd2's keep bits read by ea_attn_fused_bwd2
    give exactly the gradients of its rehashing path (no mask)."""
    from espnet_amd import hip_ops as ops
    from espnet_amd._lib import lib
    from espnet_amd.layers.common import attn_fused_bwd
    B, H, p, seed = 2, 2, 0.1, 4242
    q, k, v, _, _, _, dO = _inputs(B, H, T1, T2, False, seed=7)
    klen = torch.tensor(klens, dtype=torch.long, device=DEV)
    O, dq1, dk1, dv1, _, _ = run_fused(q, k, v, None, None, None, klen, causal, H, dO, p=p, seed=seed)
    d = H * 64
    ldm = 2 * ((T2 + 63) // 64)
    dmask = torch.empty(B * H * T1 * ldm, dtype=torch.int32, device=DEV)
    O2 = torch.empty_like(O)
    lse = torch.empty(B * H * T1, device=DEV)
    lib.ea_attn_fused_fwd2(B, H, T1, T2, 64, q.data_ptr(), d, k.data_ptr(), d, v.data_ptr(), d, 0, 0, 0, 0,
                           klen.data_ptr(), int(causal), 1 / 8, p, seed, O2.data_ptr(), d, lse.data_ptr(),
                           dmask.data_ptr(), ldm, ops.stream())
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    attn_fused_bwd(B=B, H=H, T1=T1, T2=T2, q=q, ldq=d, k=k, ldk=d, v=v, ldv=d, bu=None, bv=None, pp=None, ldp=0,
                   klen=klen, causal=causal, scale=1 / 8, p=p, seed=seed, O=O2, ldo=d, lse=lse, dO=dO, lddo=d,
                   dq=dq, lddq=d, dk=dk, lddk=d, dv=dv, lddv=d, dmask=dmask, ldm=ldm)
    torch.cuda.synchronize()
    assert torch.equal(O2, O)
    assert torch.equal(dq, dq1) and torch.equal(dk, dk1) and torch.equal(dv, dv1)


@pytest.mark.parametrize("B,H,T,klens,p,mask", [
    (2, 3, 137, [137, 100], 0.0, False),
    (3, 2, 249, [249, 200, 64], 0.1, True),
    (2, 2, 249, [249, 249], 0.1, False),
    (1, 2, 300, [300], 0.1, True),
    (2, 1, 97, [97, 1], 0.0, False),
    (2, 2, 45, [45, 30], 0.1, True),
    (2, 2, 499, [499, 331], 0.1, True),
])
def test_bwdq_pipelined_matches_original(B, H, T, klens, p, mask):
    """The pipelined dQ pass (flags bit 1: LDS-DMA one chunk ahead, bpermute gather, 64-column
    band windows, shifted 16-B dbd stores) against the original pass on the same inputs: dk,
    dv, dbd (logical columns) and the pos_bias_u partials bit for bit; dq and the pos_bias_v
    partials (d(q+v) summed over 64- instead of 96-column windows) to f32 rounding."""
    from espnet_amd import hip_ops as ops
    from espnet_amd._lib import lib
    from espnet_amd.layers.common import attn_fused_bwd
    q, k, v, u, vb, pp, dO = _inputs(B, H, T, T, True, seed=11)
    klen = torch.tensor(klens, dtype=torch.long, device=DEV)
    d, seed, scale = H * 64, 77, 1 / 8
    ldm = 2 * ((T + 63) // 64)
    dmask = torch.empty(B * H * T * ldm, dtype=torch.int32, device=DEV) if mask else None
    O = torch.empty(B, T, d, dtype=bf, device=DEV)
    lse = torch.empty(B * H * T, device=DEV)
    lib.ea_attn_fused_fwd2(B, H, T, T, 64, q.data_ptr(), d, k.data_ptr(), d, v.data_ptr(), d, u.data_ptr(),
                           vb.data_ptr(), pp.data_ptr(), d, klen.data_ptr(), 0, scale, p, seed, O.data_ptr(), d,
                           lse.data_ptr(), 0 if dmask is None else dmask.data_ptr(), ldm, ops.stream())
    nqb = (T + 63) // 64
    out = {}
    for v2 in (False, True):
        sh, ld = dbd_layout(T, v2)
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        dbd = torch.full((H * B * T * ld,), float("nan"), dtype=bf, device=DEV)
        part = torch.full((2, B * nqb, d), float("nan"), device=DEV)
        qv = torch.empty(B, T, d, dtype=bf, device=DEV)
        attn_fused_bwd(B=B, H=H, T1=T, T2=T, q=q, ldq=d, k=k, ldk=d, v=v, ldv=d, bu=u, bv=vb, pp=pp, ldp=d,
                       klen=klen, causal=False, scale=scale, p=p, seed=seed, O=O, ldo=d, lse=lse, dO=dO, lddo=d,
                       dq=dq, lddq=d, dk=dk, lddk=d, dv=dv, lddv=d, dbd=dbd, ldbd=ld, part=part, ldpart=d,
                       qv_out=qv, ldqv=d, dmask=dmask, ldm=ldm, flags=1 | (2 if v2 else 4))
        torch.cuda.synchronize()
        band, outside = band_view(dbd, H, B, T, v2)
        out[v2] = (dq, dk, dv, band, outside, part, qv)
    (dq1, dk1, dv1, b1, o1, p1, qv1), (dq2, dk2, dv2, b2, o2, p2, qv2) = out[False], out[True]
    assert torch.equal(dk1, dk2) and torch.equal(dv1, dv2) and torch.equal(qv1, qv2)
    assert torch.equal(b1, b2)
    assert o2.numel() == 0 or float(o2.float().abs().max()) == 0.0
    assert torch.equal(p1[0], p2[0])
    assert _rel(dq2, dq1) < 2e-3
    assert float((dq2.float() - dq1.float()).abs().max()) <= 2e-2 * float(dq1.float().abs().max())
    assert _rel(p2[1], p1[1]) < 1e-4


@pytest.mark.parametrize("B,H,T1,T2,rel,causal,klens,p", [
    (3, 2, 249, 249, True, False, [249, 200, 64], 0.1),
    (2, 3, 137, 137, True, False, [137, 100], 0.0),
    (1, 2, 300, 300, True, False, [300], 0.1),
    (2, 2, 45, 45, False, True, [45, 30], 0.1),
    (2, 1, 41, 300, False, False, [300, 131], 0.0),
    (1, 1, 5, 5, True, False, [5], 0.1),
    (2, 2, 499, 499, True, False, [499, 331], 0.1),
    (2, 1, 81, 499, False, False, [499, 330], 0.0),
])
def test_fwd_pipelined_matches_original(B, H, T1, T2, rel, causal, klens, p, monkeypatch):
    """The pipelined forward (LDS-DMA one chunk ahead, bpermute BD gather, Pd^T image) is the
    original forward's arithmetic in the same order: O, lse and the keep bits bit for bit."""
    from espnet_amd import hip_ops as ops
    from espnet_amd._lib import lib
    q, k, v, u, vb, pp, _ = _inputs(B, H, T1, T2, rel, seed=21)
    klen = torch.tensor(klens, dtype=torch.long, device=DEV)
    d = H * 64
    ldm = 2 * ((T2 + 63) // 64)
    ptr = lambda t: 0 if t is None else t.data_ptr()  # noqa: E731
    out = []
    for v1 in ("1", "0"):
        monkeypatch.setenv("EA_ATTN_FWD_V1", v1)
        O = torch.empty(B, T1, d, dtype=bf, device=DEV)
        lse = torch.empty(B * H * T1, device=DEV)
        dmask = torch.zeros(B * H * T1 * ldm, dtype=torch.int32, device=DEV)
        lib.ea_attn_fused_fwd2(B, H, T1, T2, 64, q.data_ptr(), d, k.data_ptr(), d, v.data_ptr(), d, ptr(u),
                               ptr(vb), ptr(pp), d, klen.data_ptr(), int(causal), 1 / 8, p, 5, O.data_ptr(), d,
                               lse.data_ptr(), dmask.data_ptr() if p > 0 else 0, ldm, ops.stream())
        torch.cuda.synchronize()
        out.append((O, lse, dmask))
    (O1, l1, m1), (O2, l2, m2) = out
    assert torch.equal(O1, O2) and torch.equal(l1, l2) and torch.equal(m1, m2)


@pytest.mark.parametrize("B,H,T1,T2,rel,causal,klens,p,mask", [
    (3, 2, 249, 249, True, False, [249, 200, 64], 0.1, True),
    (2, 3, 137, 137, True, False, [137, 100], 0.0, False),
    (1, 2, 300, 300, True, False, [300], 0.1, False),
    (2, 2, 45, 45, False, True, [45, 30], 0.1, True),
    (2, 1, 41, 300, False, False, [300, 131], 0.0, False),
    (1, 1, 5, 5, True, False, [5], 0.1, True),
    (2, 2, 499, 499, True, False, [499, 331], 0.1, True),
    (1, 1, 499, 499, False, True, [499], 0.1, False),
])
def test_bwdkv_pipelined_matches_original(B, H, T1, T2, rel, causal, klens, p, mask, monkeypatch):
    """The pipelined dK/dV pass (LDS-DMA one query tile ahead, per-wave BD tiles gathered by
    bpermute) recomputes the same values in the same MFMA order: dK, dV bit for bit."""
    from espnet_amd import hip_ops as ops
    from espnet_amd._lib import lib
    from espnet_amd.layers.common import attn_fused_bwd
    q, k, v, u, vb, pp, dO = _inputs(B, H, T1, T2, rel, seed=31)
    klen = torch.tensor(klens, dtype=torch.long, device=DEV)
    d = H * 64
    ldm = 2 * ((T2 + 63) // 64)
    ptr = lambda t: 0 if t is None else t.data_ptr()  # noqa: E731
    O = torch.empty(B, T1, d, dtype=bf, device=DEV)
    lse = torch.empty(B * H * T1, device=DEV)
    dmask = torch.zeros(B * H * T1 * ldm, dtype=torch.int32, device=DEV) if mask else None
    lib.ea_attn_fused_fwd2(B, H, T1, T2, 64, q.data_ptr(), d, k.data_ptr(), d, v.data_ptr(), d, ptr(u), ptr(vb),
                           ptr(pp), d, klen.data_ptr(), int(causal), 1 / 8, p, 9, O.data_ptr(), d, lse.data_ptr(),
                           ptr(dmask), ldm, ops.stream())
    out = []
    for v1 in ("1", "0"):
        monkeypatch.setenv("EA_ATTN_BWDKV_V1", v1)
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        attn_fused_bwd(B=B, H=H, T1=T1, T2=T2, q=q, ldq=d, k=k, ldk=d, v=v, ldv=d, bu=u, bv=vb, pp=pp, ldp=d,
                       klen=klen, causal=causal, scale=1 / 8, p=p, seed=9, O=O, ldo=d, lse=lse, dO=dO, lddo=d,
                       dq=dq, lddq=d, dk=dk, lddk=d, dv=dv, lddv=d, dmask=dmask, ldm=ldm)
        torch.cuda.synchronize()
        out.append((dq, dk, dv))
    (dq1, dk1, dv1), (dq2, dk2, dv2) = out
    assert torch.equal(dq1, dq2) and torch.equal(dk1, dk2) and torch.equal(dv1, dv2)


