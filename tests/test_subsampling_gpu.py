"""Conv2dSubsampling on the AMP (bf16) path: the implicit-GEMM route (conv1 direct into the
phase-split x1p; conv2 forward / per-parity-class input gradient / weight gradient as
gathered LDS-DMA GEMMs; fused conv1 weight gradient) against the im2col route and against
the exact-f32 route, forward output and every parameter gradient
(espnet/nets/pytorch_backend/transformer/subsampling.py:46-91)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(C, B, T, implicit, cd, seed=0):
    from espnet_amd.arena import ParamArena
    from espnet_amd.layers import subsampling as S
    torch.manual_seed(seed)
    sub = S.Conv2dSubsampling(80, C, 0.0)
    dev = torch.device("cuda", 0)
    arena = ParamArena(sub, dev, [], shadow_dtype=cd)
    sub.bind(arena, "", cd)
    sub._anchor = torch.zeros(1, device=dev, requires_grad=True)
    sub.train()
    g = torch.Generator().manual_seed(seed + 1)
    feats = torch.randn(B, T, 80, generator=g).to(dev)
    old = S._implicit_ok
    S._implicit_ok = (lambda cd_, C_: old(cd_, C_)) if implicit else (lambda cd_, C_: False)
    try:
        y = sub(feats, 0)
        gy = torch.randn(y.shape, generator=g).to(dev)
        y.backward(gy)
    finally:
        S._implicit_ok = old
    torch.cuda.synchronize()
    grads = {k: p.grad.detach().clone() for k, p in sub.named_parameters()}
    return y.detach().float(), grads


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


@pytest.mark.parametrize("C,B,T", [(64, 3, 61), (256, 2, 97), (512, 2, 131)])
def test_implicit_bf16_matches_im2col_and_f32(C, B, T):
    y_i, g_i = _run(C, B, T, True, torch.bfloat16)
    y_c, g_c = _run(C, B, T, False, torch.bfloat16)
    y_f, g_f = _run(C, B, T, False, torch.float32)
    # bf16 operands, f32 accumulation: both bf16 routes sit at bf16 distance from exact f32;
    # the implicit route computes conv1 in f32 (the im2col route rounds x and w1 to bf16
    # first), so it is at least as close to f32
    e_i, e_c = _rel(y_i, y_f), _rel(y_c, y_f)
    assert e_i < 1e-2 and e_i <= e_c * 1.5, (e_i, e_c)
    assert _rel(y_i, y_c) < 1e-2
    # weight/bias gradients sum bf16-rounded upstream gradients over every pixel: a few %
    # from f32 on both bf16 routes (measured 4-5% at C=64); the implicit route must not be
    # worse than the im2col route
    for k in g_f:
        ei, ec = _rel(g_i[k], g_f[k]), _rel(g_c[k], g_f[k])
        assert ei < 1e-1 and ei <= ec * 1.5 + 1e-3, (k, ei, ec)


@pytest.mark.parametrize("C,B,T", [(64, 3, 61), (512, 2, 131), (256, 4, 300)])
def test_implicit_pipe_kernel_matches_lds_kernel(C, B, T):
    """The three conv2 gather modes (forward, per-class input gradient, split-K weight
    gradient) on the ping-pong kernel (gemm_pipe) against gemm_bf16_lds, both on 256x256
    tiles: the same K order and the same split, so the results agree to the bit."""
    from espnet_amd._lib import GEMM_PIPE, lib
    from espnet_amd.layers import subsampling as S
    lib.ea_gemm_set_tile(256, 256)
    fuse = S.FUSE_CONV1_WGRAD
    S.FUSE_CONV1_WGRAD = False  # the fused conv1 epilogue exists on the ping-pong kernel only
    try:
        lib.ea_gemm_set_pipe(0)
        y0, g0 = _run(C, B, T, True, torch.bfloat16)
        lib.ea_gemm_set_pipe(1)
        y1, g1 = _run(C, B, T, True, torch.bfloat16)
    finally:
        lib.ea_gemm_set_tile(0, 0)
        lib.ea_gemm_set_pipe(GEMM_PIPE)
        S.FUSE_CONV1_WGRAD = fuse
    assert torch.equal(y0, y1)
    for k in g0:
        assert torch.equal(g0[k], g1[k]), k


@pytest.mark.parametrize("C,B,T", [(64, 3, 61), (512, 2, 131), (256, 4, 300)])
def test_fused_conv1_wgrad_matches_unfused(C, B, T):
    """ea_gemm_conv_w1: conv1's weight / bias gradient from the conv2 input-gradient tiles'
    epilogues equals the unfused route (dx1 stored in bf16, then ea_conv1_wgrad) up to the
    f32 summation order (the masked gradient is bf16-rounded in both; the input patches enter
    the MFMA as bf16 hi + lo halves); every other output is bit-identical."""
    from espnet_amd.layers import subsampling as S
    fuse, bits = S.FUSE_CONV1_WGRAD, S.CONV1_POS_BITS
    try:
        S.FUSE_CONV1_WGRAD = False
        y0, g0 = _run(C, B, T, True, torch.bfloat16)
        S.FUSE_CONV1_WGRAD, S.CONV1_POS_BITS = True, False  # mask from the bf16 x1p rows
        y2, g2 = _run(C, B, T, True, torch.bfloat16)
        S.CONV1_POS_BITS = True  # mask from ea_conv1_fwd2's support bits
        y1, g1 = _run(C, B, T, True, torch.bfloat16)
    finally:
        S.FUSE_CONV1_WGRAD, S.CONV1_POS_BITS = fuse, bits
    assert torch.equal(y0, y1) and torch.equal(y2, y1)
    for k in g1:
        assert torch.equal(g1[k], g2[k]), k  # same mask, same arithmetic
    for k in g0:
        if k.startswith("conv.0."):
            # two f32 summation orders over ~10^5 pixels whose products largely cancel
            # (measured 3.3e-5 at C=512)
            assert _rel(g1[k], g0[k]) < 2e-4, (k, _rel(g1[k], g0[k]))
        else:
            assert torch.equal(g0[k], g1[k]), k


@pytest.mark.parametrize("C,B,T", [(64, 3, 61), (512, 2, 131), (256, 4, 300), (512, 32, 1000)])
def test_merged_dgrad_classes_bit_identical(C, B, T):
    """ea_gemm_conv_w1b_all: the four parity classes of the conv2 input gradient (with the fused
    conv1 weight gradient) in ONE launch, longest K first, equal bit for bit to the four
    per-class launches — same tiles, same arithmetic, same partial-tile layout; the C3 shape
    (B=32, T=1000) included."""
    from espnet_amd.layers import subsampling as S
    merged = S.MERGED_DGRAD
    try:
        S.MERGED_DGRAD = False
        y0, g0 = _run(C, B, T, True, torch.bfloat16)
        S.MERGED_DGRAD = True
        y1, g1 = _run(C, B, T, True, torch.bfloat16)
    finally:
        S.MERGED_DGRAD = merged
    assert torch.equal(y0, y1)
    for k in g0:
        assert torch.equal(g0[k], g1[k]), k


@pytest.mark.gpu
@pytest.mark.parametrize("C,B,T", [(64, 2, 67), (256, 3, 131), (512, 32, 1000)])
def test_dgrad_kmajor_weight_bit_identical(C, B, T):
    """The merged conv2 input gradient reading conv2's weight K-major (W2k [ci][tap][co], ldb =
    9C: b128 fragment reads) equals the W2t [tap][co][ci] (transposed-read) launch bit for bit:
    the same products summed in the same order."""
    from espnet_amd.layers import subsampling as S
    prev = S.DGRAD_KMAJOR
    try:
        S.DGRAD_KMAJOR = False
        y0, g0 = _run(C, B, T, True, torch.bfloat16)
        S.DGRAD_KMAJOR = True
        y1, g1 = _run(C, B, T, True, torch.bfloat16)
    finally:
        S.DGRAD_KMAJOR = prev
    assert torch.equal(y0, y1)
    for k in g0:
        assert torch.equal(g0[k], g1[k]), k
