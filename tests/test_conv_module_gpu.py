"""Conformer convolution module pieces (conformer/convolution.py:38-79) on the C-ABI:
BatchNorm (training statistics) + Swish backward (ea_batchnorm_bwd) and the depthwise Conv1d
backward with the GLU backward fused into its input-gradient store (ea_dwconv_glu_bwd), each
against a plain fp64 torch reference; the fused kernel also against the two-kernel path
(ea_dwconv_bwd + ea_glu_bwd): the same arithmetic, equal up to last-ulp differences of the tap
sums where the compiler contracts them differently."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("rows,C", [(7968, 512), (15968, 512), (100, 64), (37, 256)])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_batchnorm_swish_bwd_vs_fp64(rows, C, dt):
    from espnet_amd import hip_ops as ops
    from espnet_amd.layers.common import ACT_SWISH
    g = torch.Generator().manual_seed(rows + C)
    y = (torch.randn(rows, C, generator=g) * 2 + 0.5).cuda()
    gamma = (torch.rand(C, generator=g) + 0.5).cuda()
    beta = (torch.randn(C, generator=g) * 0.1).cuda()
    mean = torch.empty(C, device="cuda")
    rstd = torch.empty(C, device="cuda")
    rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    nbt = torch.zeros(1, dtype=torch.int64, device="cuda")
    z = torch.empty(rows, C, dtype=dt, device="cuda")
    ops.batchnorm_fwd(y, gamma, beta, mean, rstd, rm, rv, nbt, z, True, ACT_SWISH, eps=1e-5, momentum=0.1)
    dz = torch.randn(rows, C, generator=g).to(dt).cuda()
    dy = torch.empty(rows, C, device="cuda")
    pg = torch.randn(2 * C, generator=g).cuda()
    dparams = pg.clone()
    ops.batchnorm_bwd(dz, y, mean, rstd, gamma, beta, ACT_SWISH, dy, dparams[:C], dparams[C:])
    torch.cuda.synchronize()
    yr = y.double().cpu().requires_grad_(True)
    gr = gamma.double().cpu().requires_grad_(True)
    br = beta.double().cpu().requires_grad_(True)
    mu = yr.mean(0)
    var = yr.var(0, unbiased=False)
    h = (yr - mu) / torch.sqrt(var + 1e-5) * gr + br
    zr = h * torch.sigmoid(h)
    zr.backward(dz.double().cpu())
    torch.testing.assert_close(dy.double().cpu(), yr.grad, atol=2e-4, rtol=1e-4)
    torch.testing.assert_close(dparams[:C].double().cpu(), pg[:C].double().cpu() + gr.grad, atol=2e-3, rtol=1e-4)
    torch.testing.assert_close(dparams[C:].double().cpu(), pg[C:].double().cpu() + br.grad, atol=2e-3, rtol=1e-4)


@pytest.mark.parametrize("B,T,C,K", [(32, 249, 512, 31), (32, 499, 512, 31), (3, 37, 64, 31), (2, 70, 128, 15),
                                     (4, 20, 64, 3)])
def test_dwconv_glu_bwd_fused(B, T, C, K):
    from espnet_amd._lib import lib
    from espnet_amd import hip_ops as ops
    g = torch.Generator().manual_seed(B * T + C + K)
    N = B * T
    g2 = torch.randn(N, 2 * C, generator=g).to(torch.bfloat16).cuda()
    a, gate = g2.float()[:, :C], g2.float()[:, C:]
    glu = (a * torch.sigmoid(gate)).contiguous()  # the forward's f32 GLU output (the conv input)
    w = (torch.randn(C, K, generator=g) * 0.2).cuda()
    dy = torch.randn(N, C, generator=g).cuda()
    ws = torch.empty(B * ((T + 31) // 32) * C * (K + 1) + 1024, device="cuda")
    st = ops.stream()
    # two-kernel path
    dglu = torch.empty(N, C, device="cuda")
    dw0 = torch.zeros(C, K, device="cuda")
    db0 = torch.zeros(C, device="cuda")
    assert lib.ea_dwconv_bwd(B, T, C, K, glu.data_ptr(), w.data_ptr(), dy.data_ptr(), dglu.data_ptr(), dw0.data_ptr(),
                             db0.data_ptr(), 1, ws.data_ptr(), ws.numel(), st) == 0
    dg2_0 = torch.empty(N, 2 * C, dtype=torch.bfloat16, device="cuda")
    assert lib.ea_glu_bwd(N, C, g2.data_ptr(), ops.dt(g2), dglu.data_ptr(), dg2_0.data_ptr(), st) == 0
    # fused
    dg2 = torch.empty(N, 2 * C, dtype=torch.bfloat16, device="cuda")
    dw = torch.zeros(C, K, device="cuda")
    db = torch.zeros(C, device="cuda")
    assert lib.ea_dwconv_glu_bwd(B, T, C, K, glu.data_ptr(), w.data_ptr(), dy.data_ptr(), g2.data_ptr(),
                                 dg2.data_ptr(), dw.data_ptr(), db.data_ptr(), 1, ws.data_ptr(), ws.numel(), st) == 0
    # dw / dbias adjacent (the parameter arena's layout): one reduction, the same sums
    pa = torch.zeros(C * K + C, device="cuda")
    dg2a = torch.empty(N, 2 * C, dtype=torch.bfloat16, device="cuda")
    assert lib.ea_dwconv_glu_bwd(B, T, C, K, glu.data_ptr(), w.data_ptr(), dy.data_ptr(), g2.data_ptr(),
                                 dg2a.data_ptr(), pa.data_ptr(), pa[C * K:].data_ptr(), 1, ws.data_ptr(), ws.numel(),
                                 st) == 0
    torch.cuda.synchronize()
    assert torch.equal(pa[:C * K].view(C, K), dw) and torch.equal(pa[C * K:], db)
    assert torch.equal(dg2a.view(torch.int16), dg2.view(torch.int16))
    # the same arithmetic as the two-kernel path; the tap sums may round differently where the
    # compiler contracts them differently (last-ulp differences, visible only where the 31-tap sum
    # cancels to ~1e-7 of its terms): a handful of elements within one bf16 ulp or 1e-6
    bad = dg2.view(torch.int16) != dg2_0.view(torch.int16)
    assert int(bad.sum()) <= max(4, bad.numel() // 100000)
    torch.testing.assert_close(dg2.float(), dg2_0.float(), atol=1e-6, rtol=8e-3)
    torch.testing.assert_close(dw, dw0, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(db, db0, atol=1e-5, rtol=1e-5)
    # fp64 reference: y = conv1d(glu) per utterance (zero padding (K-1)/2), glu = a * sigmoid(b)
    g2r = g2.double().cpu().requires_grad_(True)
    ar, br_ = g2r[:, :C], g2r[:, C:]
    xr = (ar * torch.sigmoid(br_)).view(B, T, C).transpose(1, 2)
    wr = w.double().cpu().requires_grad_(True)
    bias = torch.zeros(C, dtype=torch.float64, requires_grad=True)
    yr = torch.nn.functional.conv1d(xr, wr.view(C, 1, K), bias, padding=(K - 1) // 2, groups=C)
    yr.backward(dy.double().cpu().view(B, T, C).transpose(1, 2))
    torch.testing.assert_close(dg2.double().cpu(), g2r.grad, atol=3e-2, rtol=1e-2)
    torch.testing.assert_close(dw.double().cpu(), wr.grad, atol=2e-2, rtol=1e-3)
    torch.testing.assert_close(db.double().cpu(), bias.grad, atol=2e-3, rtol=1e-4)


@pytest.mark.parametrize("B,T,C,K", [(32, 249, 512, 31), (3, 37, 64, 31), (2, 70, 128, 15), (4, 20, 64, 3)])
def test_dwconv_glu_in_conv(B, T, C, K):
    """The depthwise conv of glu(g2) computed in the tile loaders (no stored f32 GLU activation):
    ea_dwconv_fwd_glu vs ea_glu_fwd + ea_dwconv_fwd, and ea_dwconv_glu_bwd with x = NULL vs with
    the stored activation — the same conv-input values (bit-identical glu), tap sums equal up to
    last-ulp contraction differences; and the forward vs fp64."""
    from espnet_amd._lib import lib
    from espnet_amd import hip_ops as ops
    g = torch.Generator().manual_seed(7 * B + T + C + K)
    N = B * T
    g2 = torch.randn(N, 2 * C, generator=g).to(torch.bfloat16).cuda()
    w = (torch.randn(C, K, generator=g) * 0.2).cuda()
    bias = torch.randn(C, generator=g).cuda()
    dy = torch.randn(N, C, generator=g).cuda()
    st = ops.stream()
    glu = torch.empty(N, C, device="cuda")
    assert lib.ea_glu_fwd(N, C, g2.data_ptr(), ops.dt(g2), glu.data_ptr(), 0, st) == 0
    y0 = torch.empty(N, C, device="cuda")
    assert lib.ea_dwconv_fwd(B, T, C, K, glu.data_ptr(), w.data_ptr(), bias.data_ptr(), y0.data_ptr(), st) == 0
    y = torch.empty(N, C, device="cuda")
    assert lib.ea_dwconv_fwd_glu(B, T, C, K, g2.data_ptr(), w.data_ptr(), bias.data_ptr(), y.data_ptr(), st) == 0
    ws = torch.empty(B * ((T + 31) // 32) * C * (K + 1) + 1024, device="cuda")
    outs = []
    for x in (glu.data_ptr(), None):
        dg2 = torch.empty(N, 2 * C, dtype=torch.bfloat16, device="cuda")
        dw = torch.zeros(C, K, device="cuda")
        db = torch.zeros(C, device="cuda")
        assert lib.ea_dwconv_glu_bwd(B, T, C, K, x, w.data_ptr(), dy.data_ptr(), g2.data_ptr(), dg2.data_ptr(),
                                     dw.data_ptr(), db.data_ptr(), 1, ws.data_ptr(), ws.numel(), st) == 0
        outs.append((dg2, dw, db))
    torch.cuda.synchronize()
    torch.testing.assert_close(y, y0, atol=1e-5, rtol=1e-5)
    (a0, w0, b0), (a1, w1, b1) = outs
    torch.testing.assert_close(a1.float(), a0.float(), atol=1e-6, rtol=8e-3)
    torch.testing.assert_close(w1, w0, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(b1, b0, atol=1e-5, rtol=1e-5)
    g2r = g2.double().cpu()
    xr = (g2r[:, :C] * torch.sigmoid(g2r[:, C:])).view(B, T, C).transpose(1, 2)
    yr = torch.nn.functional.conv1d(xr, w.double().cpu().view(C, 1, K), bias.double().cpu(), padding=(K - 1) // 2,
                                    groups=C)
    torch.testing.assert_close(y.double().cpu(), yr.transpose(1, 2).reshape(N, C), atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("B,T,C,K", [(32, 249, 512, 31), (3, 37, 64, 31), (4, 20, 64, 3)])
def test_bn_stats_in_dwconv_fwd(B, T, C, K):
    """ea_dwconv_fwd_glu_stats + ea_batchnorm_fwd_parts (the BatchNorm statistics from the conv's
    own tiles, shifted by the conv bias) vs ea_dwconv_fwd_glu + ea_batchnorm_fwd, and the batch
    mean / variance vs fp64."""
    import ctypes
    from espnet_amd._lib import lib
    from espnet_amd import hip_ops as ops
    from espnet_amd.layers.common import ACT_SWISH
    g = torch.Generator().manual_seed(11 * B + T + C + K)
    N = B * T
    g2 = torch.randn(N, 2 * C, generator=g).to(torch.bfloat16).cuda()
    w = (torch.randn(C, K, generator=g) * 0.2).cuda()
    bias = torch.randn(C, generator=g).cuda()
    gamma = (torch.rand(C, generator=g) + 0.5).cuda()
    beta = (torch.randn(C, generator=g) * 0.1).cuda()
    st = ops.stream()
    res = []
    for fused in (False, True):
        y = torch.empty(N, C, device="cuda")
        mean, rstd = torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
        rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
        nbt = torch.zeros(1, dtype=torch.int64, device="cuda")
        z = torch.empty(N, C, dtype=torch.bfloat16, device="cuda")
        if fused:
            npart = ctypes.c_int(0)
            assert lib.ea_dwconv_stats_parts(B, T, ctypes.addressof(npart)) == 0
            part = torch.empty(npart.value * 2 * C, device="cuda")
            assert lib.ea_dwconv_fwd_glu_stats(B, T, C, K, g2.data_ptr(), w.data_ptr(), bias.data_ptr(), y.data_ptr(),
                                               part.data_ptr(), st) == 0
            assert lib.ea_batchnorm_fwd_parts(N, C, y.data_ptr(), part.data_ptr(), npart.value, bias.data_ptr(),
                                              gamma.data_ptr(), beta.data_ptr(), 1e-5, 0.1, mean.data_ptr(),
                                              rstd.data_ptr(), rm.data_ptr(), rv.data_ptr(), nbt.data_ptr(), ACT_SWISH,
                                              z.data_ptr(), ops.dt(z), st) == 0
        else:
            assert lib.ea_dwconv_fwd_glu(B, T, C, K, g2.data_ptr(), w.data_ptr(), bias.data_ptr(), y.data_ptr(),
                                         st) == 0
            ops.batchnorm_fwd(y, gamma, beta, mean, rstd, rm, rv, nbt, z, True, ACT_SWISH, eps=1e-5, momentum=0.1)
        res.append((y, mean, rstd, rm, rv, nbt, z))
    torch.cuda.synchronize()
    (y0, m0, r0, rm0, rv0, n0, z0), (y1, m1, r1, rm1, rv1, n1, z1) = res
    # (the two conv instantiations may contract the tap sums differently: last-ulp differences)
    torch.testing.assert_close(y1, y0, atol=1e-5, rtol=1e-5)
    assert int(n0) == int(n1) == 1
    for a, b_ in ((m0, m1), (r0, r1), (rm0, rm1), (rv0, rv1)):
        torch.testing.assert_close(b_, a, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(z1.float(), z0.float(), atol=2e-2, rtol=1e-2)
    yd = y0.double().cpu()
    torch.testing.assert_close(m1.double().cpu(), yd.mean(0), atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(r1.double().cpu(), 1.0 / torch.sqrt(yd.var(0, unbiased=False) + 1e-5), atol=1e-5,
                               rtol=1e-5)
