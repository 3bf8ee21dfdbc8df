"""ea_gemm (MFMA GEMM + epilogues) vs a plain PyTorch fp64 reference of the same op."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ops():
    from espnet_amd import hip_ops
    from espnet_amd import _lib
    return hip_ops, _lib


def ref_mm(A, B, a_k, b_k, M, N, K):
    a = A.double().cpu()
    b = B.double().cpu()
    a = a[:M, :K] if a_k else a[:K, :M].t()
    b = b[:N, :K].t() if b_k else b[:K, :N]
    return a @ b


def mk(shape, dtype, gen, scale=1.0):
    return (torch.randn(shape, generator=gen) * scale).to(dtype).cuda()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("a_k,b_k", [(1, 1), (1, 0), (0, 1), (0, 0)])
@pytest.mark.parametrize("MNK", [(128, 128, 64), (100, 72, 40), (257, 130, 300), (33, 260, 129)])
def test_gemm_layouts(dtype, a_k, b_k, MNK):
    ops, L = _ops()
    M, N, K = MNK
    g = torch.Generator().manual_seed(M * 7 + N + K)
    up = lambda n: (n + 7) // 8 * 8 + 8  # leading dims must be 16-B multiples
    A = mk((M, up(K)) if a_k else (K, up(M)), dtype, g)
    B = mk((N, up(K)) if b_k else (K, up(N)), dtype, g)
    C = torch.full((M, N + 3), 7.0, device="cuda")
    ops.gemm(A, B, C, M=M, N=N, K=K, a_kmajor=a_k, b_kmajor=b_k, lda=A.stride(0),
             ldb=B.stride(0), ldc=C.stride(0))
    ref = ref_mm(A, B, a_k, b_k, M, N, K)
    tol = 1e-5 if dtype == torch.float32 else 2e-3
    torch.testing.assert_close(C[:, :N].double().cpu(), ref, atol=tol * K ** 0.5, rtol=tol)
    assert (C[:, N:] == 7.0).all(), "wrote outside ldc columns"


def test_gemm_identity_asymmetric():
    ops, L = _ops()
    n = 64
    A = torch.eye(n, device="cuda")
    B = torch.arange(n * n, dtype=torch.float32, device="cuda").view(n, n) / 100.0
    C = torch.zeros(n, n, device="cuda")
    ops.gemm(A, B, C, M=n, N=n, K=n, a_kmajor=1, b_kmajor=0, lda=n, ldb=n, ldc=n)
    torch.testing.assert_close(C, B, atol=0, rtol=0)
    ops.gemm(A, B, C, M=n, N=n, K=n, a_kmajor=1, b_kmajor=1, lda=n, ldb=n, ldc=n)
    torch.testing.assert_close(C, B.t(), atol=0, rtol=0)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gemm_epilogues(dtype):
    ops, L = _ops()
    g = torch.Generator().manual_seed(3)
    M, N, K = 200, 96, 80
    x = mk((M, K), dtype, g)
    w = mk((N, K), dtype, g, 0.2)
    bias = mk((N,), torch.float32, g)
    ref = (x.double().cpu() @ w.double().cpu().t()) + bias.double().cpu()
    tol = dict(atol=1e-4, rtol=1e-4) if dtype == torch.float32 else dict(atol=3e-2, rtol=2e-2)
    # STORE with bias + post_scale, f32 out
    C = torch.empty(M, N, device="cuda")
    ops.linear(x, w, C, epi=ops.make_epi(bias=bias, post_scale=2.0))
    torch.testing.assert_close(C.double().cpu(), ref * 2.0, **tol)
    # ACT swish: aux = pre-activation, C = swish(h)
    aux = torch.empty(M, N, device="cuda", dtype=dtype)
    Ca = torch.empty(M, N, device="cuda", dtype=dtype)
    ops.linear(x, w, Ca, epi=ops.make_epi(L.EPI_ACT, bias=bias, act=L.ACT_SWISH, aux=aux))
    torch.testing.assert_close(aux.double().cpu(), ref, **tol)
    torch.testing.assert_close(Ca.double().cpu(), ref * torch.sigmoid(ref), **tol)
    # RESID: C = resid + 0.5 * v   (in place)
    R = torch.randn(M, N, generator=g).cuda()
    R0 = R.clone()
    ops.linear(x, w, R, epi=ops.make_epi(L.EPI_RESID, bias=bias, resid=R, rscale=0.5))
    torch.testing.assert_close(R.double().cpu(), R0.double().cpu() + 0.5 * ref, **tol)
    # DACT: dh = (dy . w^T...) * swish'(aux)
    Cd = torch.empty(M, N, device="cuda")
    ops.linear(x, w, Cd, epi=ops.make_epi(L.EPI_DACT, act=L.ACT_SWISH, aux=aux))
    h = aux.double().cpu()
    s = torch.sigmoid(h)
    torch.testing.assert_close(Cd.double().cpu(), (ref - bias.double().cpu()) * s * (1 + h * (1 - s)), **tol)
    # beta accumulate
    Cb = torch.ones(M, N, device="cuda")
    ops.linear(x, w, Cb, epi=ops.make_epi(beta=1.0))
    torch.testing.assert_close(Cb.double().cpu(), ref - bias.double().cpu() + 1.0, **tol)


def test_gemm_dropout_mask_consistency():
    ops, L = _ops()
    g = torch.Generator().manual_seed(5)
    M, N, K = 256, 256, 64
    x = mk((M, K), torch.float32, g)
    w = mk((N, K), torch.float32, g)
    aux = torch.empty(M, N, device="cuda")
    y = torch.empty(M, N, device="cuda")
    p = 0.25
    ops.linear(x, w, y, epi=ops.make_epi(L.EPI_ACT, act=L.ACT_NONE, aux=aux, drop_p=p, seed=1234))
    kept = (y != 0)
    frac = kept.float().mean().item()
    assert abs(frac - (1 - p)) < 0.01, frac
    torch.testing.assert_close(y[kept], aux[kept] / (1 - p))
    # backward regenerates the same mask
    d = torch.empty(M, N, device="cuda")
    ops.linear(x, w, d, epi=ops.make_epi(L.EPI_DACT, act=L.ACT_NONE, aux=aux, drop_p=p, seed=1234))
    assert torch.equal(d != 0, kept)
    # different seed -> different mask
    y2 = torch.empty(M, N, device="cuda")
    ops.linear(x, w, y2, epi=ops.make_epi(L.EPI_ACT, aux=aux, drop_p=p, seed=99))
    assert not torch.equal(y2 != 0, kept)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gemm_batched_heads(dtype):
    """scores[b,h] = q[b,:,h,:] . k[b,:,h,:]^T with (B,T,H,dk) layouts (attention)."""
    ops, L = _ops()
    g = torch.Generator().manual_seed(9)
    Bn, T, H, dk = 3, 37, 4, 64
    q = mk((Bn, T, 3 * H * dk), dtype, g)  # fused qkv rows
    k = q[:, :, H * dk:2 * H * dk]
    qq = q[:, :, :H * dk]
    S = torch.zeros(Bn, H, T, 40, device="cuda")
    ops.gemm(qq, k, S, M=T, N=T, K=dk, a_kmajor=1, b_kmajor=1, lda=3 * H * dk, ldb=3 * H * dk,
             ldc=40, batch=Bn, nh=H, sA=(T * 3 * H * dk, dk), sB=(T * 3 * H * dk, dk),
             sC=(H * T * 40, T * 40), epi=ops.make_epi(alpha=0.125))
    qr = qq.double().cpu().view(Bn, T, H, dk).transpose(1, 2)
    kr = k.double().cpu().reshape(Bn, T, H, dk).transpose(1, 2)
    ref = qr @ kr.transpose(-1, -2) * 0.125
    tol = dict(atol=1e-4, rtol=1e-4) if dtype == torch.float32 else dict(atol=5e-2, rtol=2e-2)
    torch.testing.assert_close(S[..., :T].double().cpu(), ref, **tol)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gemm_splitk_dw(dtype):
    ops, L = _ops()
    g = torch.Generator().manual_seed(4)
    R, N, K = 3000, 96, 136
    dy = mk((R, N), dtype, g)
    x = mk((R, K), dtype, g)
    dw = torch.ones(N, K, device="cuda")
    ops.linear_dw(dy, x, dw, accumulate=True)
    ref = dy.double().cpu().t() @ x.double().cpu() + 1.0
    tol = dict(atol=2e-3, rtol=1e-4) if dtype == torch.float32 else dict(atol=0.3, rtol=2e-2)
    torch.testing.assert_close(dw.double().cpu(), ref, **tol)
    dx = torch.empty(R, K, device="cuda")
    w = mk((N, K), dtype, g)
    ops.linear_dx(dy, w, dx)
    torch.testing.assert_close(dx.double().cpu(), dy.double().cpu() @ w.double().cpu(), **tol)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("a_k,b_k", [(1, 1), (1, 0), (0, 1), (0, 0)])
def test_gemm_unaligned_leading_dims(dtype, a_k, b_k):
    ops, L = _ops()
    M, N, K = 52, 50, 67
    g = torch.Generator().manual_seed(17)
    A = mk((M, K) if a_k else (K, M), dtype, g)   # ld = K or M: not 16-B multiples
    B = mk((N, K) if b_k else (K, N), dtype, g)
    C = torch.empty(M, N, device="cuda")
    ops.gemm(A, B, C, M=M, N=N, K=K, a_kmajor=a_k, b_kmajor=b_k, lda=A.stride(0), ldb=B.stride(0), ldc=N)
    tol = 1e-5 if dtype == torch.float32 else 2e-3
    torch.testing.assert_close(C.double().cpu(), ref_mm(A, B, a_k, b_k, M, N, K), atol=tol * K ** 0.5, rtol=tol)


# (bm, bn, pipe): pipe=1 routes the 256x256 tile to gemm_pipe (4-slot ring of 32-deep slices)
from espnet_amd._lib import GEMM_PIPE as PIPE_DEFAULT  # noqa: E402  (restored after each test)
# (bm, bn, pipe[, 128x128 ring slots])
TILES = [(32, 128, 0), (64, 128, 0), (128, 128, 0), (128, 128, 3), (256, 256, 0), (256, 256, 1)]


def _tile_id(t):
    return f"{t[0]}x{t[1]}{'p' * t[2]}"


@pytest.fixture
def forced_tile(request):
    ops, L = _ops()
    bm, bn, pipe = request.param[:3]
    L.lib.ea_gemm_set_tile(bm, bn)
    L.lib.ea_gemm_set_pipe(pipe)
    yield (bm, bn)
    L.lib.ea_gemm_set_tile(0, 0)
    L.lib.ea_gemm_set_pipe(PIPE_DEFAULT)


@pytest.mark.parametrize("forced_tile", TILES, indirect=True, ids=_tile_id)
@pytest.mark.parametrize("a_k,b_k", [(1, 1), (1, 0), (0, 1), (0, 0)])
@pytest.mark.parametrize("MNK", [(300, 520, 200), (513, 257, 64), (40, 300, 130), (256, 256, 128),
                                 (600, 700, 1000), (260, 300, 32)])
def test_gemm_bf16_tiles(forced_tile, a_k, b_k, MNK):
    """Every LDS-DMA tile shape (edges in M, N and a K remainder) vs fp64."""
    ops, L = _ops()
    M, N, K = MNK
    g = torch.Generator().manual_seed(M + 3 * N + 7 * K + a_k * 11 + b_k * 13)
    up = lambda n: (n + 7) // 8 * 8 + 8
    A = mk((M, up(K)) if a_k else (K, up(M)), torch.bfloat16, g)
    B = mk((N, up(K)) if b_k else (K, up(N)), torch.bfloat16, g)
    C = torch.full((M, N + 4), 7.0, device="cuda")
    ops.gemm(A, B, C, M=M, N=N, K=K, a_kmajor=a_k, b_kmajor=b_k, lda=A.stride(0),
             ldb=B.stride(0), ldc=C.stride(0), splitk=False)
    ref = ref_mm(A, B, a_k, b_k, M, N, K)
    torch.testing.assert_close(C[:, :N].double().cpu(), ref, atol=2e-3 * K ** 0.5, rtol=2e-3)
    assert (C[:, N:] == 7.0).all(), "wrote outside ldc columns"


@pytest.mark.parametrize("forced_tile", TILES, indirect=True, ids=_tile_id)
def test_gemm_bf16_tiles_epilogue_splitk(forced_tile):
    """Fused ACT epilogue and split-K dW under each tile shape."""
    ops, L = _ops()
    g = torch.Generator().manual_seed(21)
    M, N, K = 260, 384, 192
    x = mk((M, K), torch.bfloat16, g)
    w = mk((N, K), torch.bfloat16, g, 0.2)
    bias = mk((N,), torch.float32, g)
    ref = (x.double().cpu() @ w.double().cpu().t()) + bias.double().cpu()
    aux = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    Ca = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    ops.linear(x, w, Ca, epi=ops.make_epi(L.EPI_ACT, bias=bias, act=L.ACT_SWISH, aux=aux))
    tol = dict(atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(aux.double().cpu(), ref, **tol)
    torch.testing.assert_close(Ca.double().cpu(), ref * torch.sigmoid(ref), **tol)
    # dW = dY^T X over many rows (split-K path)
    R = 4000
    dy = mk((R, 96), torch.bfloat16, g)
    xx = mk((R, 160), torch.bfloat16, g)
    dw = torch.zeros(96, 160, device="cuda")
    ops.linear_dw(dy, xx, dw)
    refw = dy.double().cpu().t() @ xx.double().cpu()
    torch.testing.assert_close(dw.double().cpu(), refw, atol=2e-3 * R ** 0.5, rtol=2e-3)


@pytest.mark.parametrize("forced_tile", TILES, indirect=True, ids=_tile_id)
@pytest.mark.parametrize("mn_major", ["A", "B", "AB"])
def test_gemm_mn_major_slice_at_allocation_end(forced_tile, mn_major):
    """The bf16 decoder fault of round 3 (commit 9880edd): an MN-major operand that is a
    column-offset slice whose last row ends exactly at the end of its allocation, with
    MN % 8 != 0.  The LDS-DMA loads read whole 16-B chunks up to MN rounded to 8 (the ea_gemm
    contract in include/espnet_amd.h), so hip_ops.gemm re-homes such a view into a padded
    copy first; the product equals fp64 and values past MN never reach C (the storage after
    the slice's columns in earlier rows holds NaN)."""
    ops, L = _ops()
    bm, bn = forced_tile
    a_k = 0 if "A" in mn_major else 1
    b_k = 0 if "B" in mn_major else 1
    if bm <= 64 and not a_k:
        pytest.skip("narrow tiles take K-major A only")
    M, N, K = 173, 203, 136
    W = 512  # row stride; the slice starts at column 256 (16-B aligned)
    g = torch.Generator().manual_seed(41 + len(mn_major))

    def operand(rows, cols, kmaj):
        if kmaj:  # K-major: (rows, cols) contiguous enough
            return mk((rows, (cols + 7) // 8 * 8), torch.bfloat16, g), None
        # MN-major (K rows of MN columns): flat storage that ends at the last row's column MN
        flat = torch.full(((rows - 1) * W + 256 + cols,), float("nan"), dtype=torch.bfloat16)
        v = torch.as_strided(flat, (rows, cols), (W, 1), 256)
        v.copy_(torch.randn(rows, cols, generator=g).to(torch.bfloat16))
        flat = flat.cuda()
        return torch.as_strided(flat, (rows, cols), (W, 1), 256), flat

    A, fa = operand(K if not a_k else M, M if not a_k else K, a_k)
    B, fb = operand(K if not b_k else N, N if not b_k else K, b_k)
    for f in (fa, fb):
        if f is not None:
            assert f.untyped_storage().nbytes() >= f.numel() * 2  # the view ends at numel
    C = torch.full((M, N + 4), 7.0, device="cuda")
    before = ops.MN_TAIL_COPIES
    ops.gemm(A, B, C, M=M, N=N, K=K, a_kmajor=a_k, b_kmajor=b_k, lda=A.stride(0), ldb=B.stride(0),
             ldc=C.stride(0), splitk=False)
    torch.cuda.synchronize()
    # each MN-major view ends exactly at its storage's end (a storage's nbytes is the size
    # asked for, whatever block the caching allocator rounded it into): each is re-homed
    assert ops.MN_TAIL_COPIES - before == len(mn_major)
    ref = ref_mm(A, B, a_k, b_k, M, N, K)
    got = C[:, :N].double().cpu()
    assert torch.isfinite(got).all()
    torch.testing.assert_close(got, ref, atol=2e-3 * K ** 0.5, rtol=2e-3)
    assert (C[:, N:] == 7.0).all()


def test_mn_tail_guard_rehomes_exact_views():
    """_mn_tail_guard copies an MN-major bf16 view (MN % 8 != 0) exactly when its storage ends
    before the last row's 16-B chunk does, keeping the view's strides from the new base."""
    ops, _ = _ops()
    K, MN, W = 5, 13, 64
    flat = torch.arange((K - 1) * W + 16 + MN, dtype=torch.float32).to(torch.bfloat16).cuda()
    v = torch.as_strided(flat, (K, MN), (W, 1), 16)
    got = ops._mn_tail_guard(v, MN, K, W, (0, 0), 1, 1)
    assert got is not v and got.numel() >= (K - 1) * W + MN + 8
    torch.testing.assert_close(torch.as_strided(got, (K, MN), (W, 1), 0), v, atol=0, rtol=0)
    roomy = torch.zeros((K - 1) * W + 16 + 16, dtype=torch.bfloat16).cuda()
    v2 = torch.as_strided(roomy, (K, MN), (W, 1), 16)
    assert ops._mn_tail_guard(v2, MN, K, W, (0, 0), 1, 1) is v2
    assert ops._mn_tail_guard(v, 16, K, W, (0, 0), 1, 1) is v  # MN % 8 == 0: whole chunks


@pytest.mark.parametrize("slots", [3, 4])
@pytest.mark.parametrize("MNK", [(7968, 512, 2048), (7968, 512, 512), (300, 200, 128), (129, 520, 64),
                                 (1000, 384, 1536), (7968, 512, 64)])
def test_gemm_k128_vs_fp64(slots, MNK):
    """gemm_k128 (128x128 tile, K-major A and B, two K groups of four waves, buffer-load LDS
    ring; the N = 512 GEMMs of the C3 step) against fp64: the bench shapes and edges in M and
    N, a single K-tile, bf16 and f32 outputs, fused RESID / ACT epilogues."""
    ops, L = _ops()
    M, N, K = MNK
    g = torch.Generator().manual_seed(M + N + K + slots)
    A = mk((M, K + 8), torch.bfloat16, g)
    B = mk((N, K + 8), torch.bfloat16, g, 0.1)
    L.lib.ea_gemm_set_k128(3, slots)
    try:
        C = torch.full((M, N + 4), 7.0, device="cuda")
        ops.gemm(A, B, C, M=M, N=N, K=K, a_kmajor=1, b_kmajor=1, lda=A.stride(0), ldb=B.stride(0), ldc=C.stride(0))
        ref = ref_mm(A, B, 1, 1, M, N, K)
        torch.testing.assert_close(C[:, :N].double().cpu(), ref, atol=2e-3 * K ** 0.5, rtol=2e-3)
        assert (C[:, N:] == 7.0).all()
        bias = mk((N,), torch.float32, g)
        R = torch.randn(M, N, generator=g).cuda()
        R0 = R.clone()
        ops.gemm(A, B, R, M=M, N=N, K=K, a_kmajor=1, b_kmajor=1, lda=A.stride(0), ldb=B.stride(0), ldc=N,
                 epi=ops.make_epi(L.EPI_RESID, bias=bias, resid=R, rscale=0.5))
        torch.testing.assert_close(R.double().cpu(), R0.double().cpu() + 0.5 * (ref + bias.double().cpu()),
                                   atol=2e-3 * K ** 0.5, rtol=2e-3)
        aux = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        Ca = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        ops.gemm(A, B, Ca, M=M, N=N, K=K, a_kmajor=1, b_kmajor=1, lda=A.stride(0), ldb=B.stride(0), ldc=N,
                 epi=ops.make_epi(L.EPI_ACT, bias=bias, act=L.ACT_SWISH, aux=aux))
        h = ref + bias.double().cpu()
        torch.testing.assert_close(aux.double().cpu(), h, atol=3e-2, rtol=2e-2)
        torch.testing.assert_close(Ca.double().cpu(), h * torch.sigmoid(h), atol=3e-2, rtol=2e-2)
    finally:
        L.lib.ea_gemm_set_k128(1, 4)


def test_gemm_k128_linear_paths_match_default():
    """ea_gemm_set_k128(1) (the default): the Linear forward / input-gradient GEMMs at the C3
    token count route to gemm_k128 and agree with the 64x128 tile (mode 0) to
    bf16-accumulation-order noise."""
    ops, L = _ops()
    g = torch.Generator().manual_seed(8)
    M = 7968
    x = mk((M, 2048), torch.bfloat16, g)
    w = mk((512, 2048), torch.bfloat16, g, 0.05)
    y0 = torch.empty(M, 512, device="cuda")
    y1 = torch.empty(M, 512, device="cuda")
    L.lib.ea_gemm_set_k128(0, 4)
    try:
        ops.linear(x, w, y0)
    finally:
        L.lib.ea_gemm_set_k128(1, 4)
    ops.linear(x, w, y1)
    torch.testing.assert_close(y1, y0, atol=1e-3, rtol=1e-3)


@pytest.mark.parametrize("xchunk", [4, 1, 0])
def test_gemm_grouped_vs_fp64(xchunk):
    """ea_gemm_grouped: several (0,0)-layout f32-accumulating problems in one launch (edge
    tiles in M and N, K remainders, beta 0 / 1, longest-K-first order) vs fp64, under each
    tile -> XCD assignment (chunks of 4 / 1 tiles round-robin over the XCDs with the
    remainder past the last whole round of chunks in launch order; 0 = contiguous ranges):
    87 tiles, so every mapping has both a chunked part and a remainder."""
    ops, L = _ops()
    import ctypes
    g = torch.Generator().manual_seed(5)
    shapes = [(300, 520, 1000, 1.0), (513, 260, 64, 0.0), (40, 300, 130, 1.0), (256, 256, 7968, 1.0),
              (1024, 512, 33, 0.0), (2048, 2048, 200, 0.0)]
    probs = []
    for M, N, K, beta in sorted(shapes, key=lambda s: -s[2]):
        up = lambda n: (n + 7) // 8 * 8 + 8  # noqa: E731  (leading dims: 16-B multiples)
        A = mk((K, up(M)), torch.bfloat16, g)      # dY: K rows of M
        B = mk((K, up(N)), torch.bfloat16, g)      # X:  K rows of N
        C = torch.randn(M, N + 4, generator=g).cuda()
        C0 = C.clone()
        probs.append((A, B, C, C0, M, N, K, beta))
    arr = (L.GroupGemm * len(probs))()
    ntiles = 0
    for i, (A, B, C, C0, M, N, K, beta) in enumerate(probs):
        arr[i] = L.GroupGemm(A.data_ptr(), B.data_ptr(), C.data_ptr(), A.stride(0), B.stride(0), C.stride(0),
                             M, N, K, beta)
        ntiles += ((M + 255) // 256) * ((N + 255) // 256)
    nb = ctypes.c_long(0)
    L.lib.ea_gemm_grouped_ws_bytes(len(probs), ntiles, ctypes.addressof(nb))
    ws = torch.empty(nb.value, dtype=torch.uint8, device="cuda")
    L.lib.ea_gemm_grouped_set_xcd_chunk(xchunk)
    try:
        L.lib.ea_gemm_grouped(0, 0, len(probs), ctypes.addressof(arr), ws.data_ptr(), ws.numel(), ops.stream())
        torch.cuda.synchronize()
    finally:
        L.lib.ea_gemm_grouped_set_xcd_chunk(4)
    for A, B, C, C0, M, N, K, beta in probs:
        ref = beta * C0[:, :N].double().cpu() + ref_mm(A, B, 0, 0, M, N, K)
        torch.testing.assert_close(C[:, :N].double().cpu(), ref, atol=2e-3 * K ** 0.5, rtol=2e-3)
        assert torch.equal(C[:, N:], C0[:, N:]), "wrote outside the N columns"


def test_deferred_linear_dw_queue():
    """linear_dw inside deferred_wgrad(): nothing runs until the flush, then every queued
    weight gradient (and its post-step) matches the immediate path to f32 rounding — not bit
    for bit: the grouped full-K tile and the per-call (split-K) GEMM sum K in different orders,
    so EA_DEFER_WGRAD changes the gradient's last bits (the reduction queue, by contrast, is
    bit-exact).  The deferred path itself is deterministic: a second flush of the same queue
    reproduces its result exactly."""
    ops, L = _ops()
    g = torch.Generator().manual_seed(9)
    R = 1000
    dys = [mk((R, n), torch.bfloat16, g) for n in (96, 256, 512)]
    xs = [mk((R, k), torch.bfloat16, g) for k in (160, 512, 64)]
    want = []
    for dy, x in zip(dys, xs):
        w = torch.randn(dy.shape[1], x.shape[1], generator=g).cuda()
        imm = w.clone()
        ops.linear_dw(dy, x, imm, accumulate=True)
        want.append((w, imm))
    outs = []
    posted = torch.zeros(96, 160, device="cuda")
    with ops.deferred_wgrad() as q:
        for (dy, x), (w, _) in zip(zip(dys, xs), want):
            d = w.clone()
            outs.append(d)
            ops.linear_dw(dy, x, d, accumulate=True,
                          post=(lambda d=d: posted.copy_(d)) if d.shape == (96, 160) else None)
        assert len(q.items) == 3 if ops.DEFER_WGRAD else True
    torch.cuda.synchronize()
    for d, (_, imm) in zip(outs, want):
        torch.testing.assert_close(d, imm, atol=1e-5 * R ** 0.5, rtol=1e-5)
    torch.testing.assert_close(posted, outs[0])
    # run-to-run determinism of the deferred path
    again = []
    with ops.deferred_wgrad():
        for (dy, x), (w, _) in zip(zip(dys, xs), want):
            d = w.clone()
            again.append(d)
            ops.linear_dw(dy, x, d, accumulate=True)
    torch.cuda.synchronize()
    for a, b in zip(again, outs):
        assert torch.equal(a, b)
    # a queue over its memory budget (EA_DEFER_BUDGET_MB) launches what it holds right away
    budget = ops.DEFER_BUDGET
    ops.DEFER_BUDGET = 1
    try:
        early = []
        with ops.deferred_wgrad() as q:
            for (dy, x), (w, _) in zip(zip(dys, xs), want):
                d = w.clone()
                early.append(d)
                ops.linear_dw(dy, x, d, accumulate=True)
                assert not q.items and q.pending == 0
        torch.cuda.synchronize()
        for d, (_, imm) in zip(early, want):
            torch.testing.assert_close(d, imm, atol=1e-5 * R ** 0.5, rtol=1e-5)
    finally:
        ops.DEFER_BUDGET = budget


@pytest.mark.parametrize("MNK", [(1, 512, 512), (10, 2048, 512), (10, 512, 2048), (16, 5000, 512), (7, 1024, 512),
                                 (13, 30, 96), (3, 4999, 64)])
def test_gemm_skinny_vs_fp64(MNK):
    """gemm_skinny (M <= 16 rows: the decoder's per-step Linears; 16 x 32 blocks whose 8 waves
    split K) against fp64 with every epilogue kind, N tails (30, 4999: element-wise epilogue)
    and ldc wider than N; and equal to the tile kernels (ea_gemm_set_skinny(0)) within
    accumulation-order noise."""
    ops, L = _ops()
    M, N, K = MNK
    g = torch.Generator().manual_seed(M * 131 + N + K)
    A = mk((M, K + 8), torch.bfloat16, g)
    W = mk((N, K + 8), torch.bfloat16, g, 0.1)
    bias = mk((N + 4,), torch.float32, g)[:N]
    ref = ref_mm(A, W, 1, 1, M, N, K) + bias.double().cpu()
    tol = dict(atol=2e-3 * K ** 0.5, rtol=2e-3)
    ldc = N + 4
    C = torch.full((M, ldc), 7.0, device="cuda")
    ops.gemm(A, W, C, M=M, N=N, K=K, a_kmajor=1, b_kmajor=1, lda=A.stride(0), ldb=W.stride(0), ldc=ldc,
             epi=ops.make_epi(bias=bias))
    torch.testing.assert_close(C[:, :N].double().cpu(), ref, **tol)
    assert (C[:, N:] == 7.0).all(), "wrote outside ldc columns"
    L.lib.ea_gemm_set_skinny(0)
    try:
        C0 = torch.full((M, ldc), 7.0, device="cuda")
        ops.gemm(A, W, C0, M=M, N=N, K=K, a_kmajor=1, b_kmajor=1, lda=A.stride(0), ldb=W.stride(0), ldc=ldc,
                 epi=ops.make_epi(bias=bias))
    finally:
        L.lib.ea_gemm_set_skinny(16)
    torch.testing.assert_close(C, C0, atol=1e-4 * K ** 0.5, rtol=1e-4)
    # ACT (ReLU, pre-activation to aux) with bf16 outputs
    aux = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    Ca = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    ops.gemm(A, W, Ca, M=M, N=N, K=K, a_kmajor=1, b_kmajor=1, lda=A.stride(0), ldb=W.stride(0), ldc=N,
             epi=ops.make_epi(L.EPI_ACT, bias=bias, act=L.ACT_RELU, aux=aux))
    torch.testing.assert_close(aux.double().cpu(), ref, atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(Ca.double().cpu(), ref.clamp_min(0), atol=3e-2, rtol=2e-2)
    # RESID in place (f32 residual stream)
    R = torch.randn(M, N, generator=g).cuda()
    R0 = R.clone()
    ops.gemm(A, W, R, M=M, N=N, K=K, a_kmajor=1, b_kmajor=1, lda=A.stride(0), ldb=W.stride(0), ldc=N,
             epi=ops.make_epi(L.EPI_RESID, bias=bias, resid=R, rscale=1.0))
    torch.testing.assert_close(R.double().cpu(), R0.double().cpu() + ref, **tol)


@pytest.mark.parametrize("a_k,b_k", [(1, 1), (1, 0), (0, 1)])
@pytest.mark.parametrize("MNK", [(7968, 512, 2048), (4100, 1536, 512), (4096, 200, 72)])
@pytest.mark.parametrize("out", [torch.bfloat16, torch.float32])
def test_gemm_plain_vs_fp64(a_k, b_k, MNK, out):
    """Plain products (alpha / beta, no other epilogue: the Linear input gradients) with every
    operand layout the host mirror issues, bf16 and f32 outputs, ldc wider than N, and the same
    call with a bias — all on the library's own MFMA kernels, against fp64."""
    ops, L = _ops()
    M, N, K = MNK
    g = torch.Generator().manual_seed(M + N + K + a_k * 2 + b_k)
    up = lambda n: (n + 7) // 8 * 8 + 8  # noqa: E731
    A = mk((M, up(K)) if a_k else (K, up(M)), torch.bfloat16, g)
    B = mk((N, up(K)) if b_k else (K, up(N)), torch.bfloat16, g, 0.1)
    ref = ref_mm(A, B, a_k, b_k, M, N, K)
    tol = dict(atol=2e-3 * K ** 0.5, rtol=2e-2 if out == torch.bfloat16 else 2e-3)
    C = torch.full((M, N + 8), 7.0, device="cuda", dtype=out)
    ops.gemm(A, B, C, M=M, N=N, K=K, a_kmajor=a_k, b_kmajor=b_k, lda=A.stride(0), ldb=B.stride(0),
             ldc=C.stride(0), epi=ops.make_epi(alpha=0.5))
    torch.testing.assert_close(C[:, :N].double().cpu(), 0.5 * ref, **tol)
    assert (C[:, N:] == 7.0).all(), "wrote outside ldc columns"
    C0 = C.clone()
    ops.gemm(A, B, C, M=M, N=N, K=K, a_kmajor=a_k, b_kmajor=b_k, lda=A.stride(0), ldb=B.stride(0),
             ldc=C.stride(0), epi=ops.make_epi(beta=1.0))
    torch.testing.assert_close(C[:, :N].double().cpu(), C0[:, :N].double().cpu() + ref, **tol)
    bias = mk((N,), torch.float32, g)
    Cb = torch.empty(M, N, device="cuda", dtype=out)
    ops.gemm(A, B, Cb, M=M, N=N, K=K, a_kmajor=a_k, b_kmajor=b_k, lda=A.stride(0), ldb=B.stride(0), ldc=N,
             epi=ops.make_epi(bias=bias))
    torch.testing.assert_close(Cb.double().cpu(), ref + bias.double().cpu(), **tol)


@pytest.mark.parametrize("MNK", [(10, 1536, 512), (10, 2048, 512), (16, 5000, 512), (3, 40, 96), (7, 512, 2048)])
def test_gemm_ln_vs_fp64(MNK):
    """ea_gemm_ln (LayerNorm of f32 rows computed inside the few-row GEMM, normalised rows
    rounded to bf16 as the unfused LayerNorm stores them): against fp64 LayerNorm -> bf16 ->
    GEMM, and equal to the unfused pair (ea_layernorm_fwd + ea_gemm) within accumulation noise."""
    ops, L = _ops()
    M, N, K = MNK
    g = torch.Generator().manual_seed(M * 5 + N + K)
    x = (torch.randn(M, K + 4, generator=g) * 3 + 1).cuda()[:, :K]
    gam = (torch.rand(K, generator=g) + 0.5).cuda()
    bet = torch.randn(K, generator=g).cuda() * 0.1
    W = mk((N, K + 8), torch.bfloat16, g, 0.1)[:, :K]
    bias = mk((N,), torch.float32, g)
    xd = x.double().cpu()
    xn = (xd - xd.mean(1, keepdim=True)) / torch.sqrt(xd.var(1, unbiased=False, keepdim=True) + 1e-12)
    xn = (xn * gam.double().cpu() + bet.double().cpu()).to(torch.bfloat16).double()
    ref = xn @ W.double().cpu().t() + bias.double().cpu()
    C = torch.full((M, N + 4), 7.0, device="cuda")
    ops.linear_ln(x, gam, bet, W, C[:, :N], epi=ops.make_epi(bias=bias))
    torch.testing.assert_close(C[:, :N].double().cpu(), ref, atol=2e-3 * K ** 0.5, rtol=2e-3)
    assert (C[:, N:] == 7.0).all()
    if K > 1024:
        return  # (the unfused LayerNorm kernel takes d <= 1024)
    xn_dev = torch.empty(M, K, device="cuda", dtype=torch.bfloat16)
    ops.layernorm_fwd(x, gam, bet, xn_dev, torch.empty(M, device="cuda"), torch.empty(M, device="cuda"))
    C0 = torch.empty(M, N, device="cuda")
    ops.linear(xn_dev, W, C0, epi=ops.make_epi(bias=bias))
    torch.testing.assert_close(C[:, :N], C0, atol=2e-2, rtol=1e-2)


