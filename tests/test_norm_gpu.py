"""LayerNorm C-ABI (ea_layernorm_fwd / ea_layernorm_bwd) vs a plain fp64 torch LayerNorm
(eps 1e-12, transformer/layer_norm.py): the vectorised one-pass kernels (d % 8 == 0) and
the generic row kernels (other d), f32 and bf16 outputs / incoming gradients."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("rows,d", [(7968, 512), (1312, 512), (333, 1024), (257, 256), (100, 80), (65, 100)])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_layernorm_fwd_bwd(rows, d, dt):
    from espnet_amd import hip_ops as ops
    g = torch.Generator().manual_seed(rows + d)
    x = (torch.randn(rows, d, generator=g) * 3 + 1).cuda()
    gamma = (torch.rand(d, generator=g) + 0.5).cuda()
    beta = torch.randn(d, generator=g).cuda()
    dy = torch.randn(rows, d, generator=g).to(dt).cuda()
    y = torch.empty(rows, d, dtype=dt, device="cuda")
    mu = torch.empty(rows, device="cuda")
    rs = torch.empty(rows, device="cuda")
    ops.layernorm_fwd(x, gamma, beta, y, mu, rs)
    dx0 = torch.randn(rows, d, generator=g).cuda()
    dx = dx0.clone()
    pg = torch.randn(2 * d, generator=g).cuda()
    dparams = pg.clone()
    ops.layernorm_bwd(dy, x, gamma, mu, rs, dx, dparams[:d], dparams[d:], accumulate=True)
    torch.cuda.synchronize()
    xr = x.double().cpu().requires_grad_(True)
    gr = gamma.double().cpu().requires_grad_(True)
    br = beta.double().cpu().requires_grad_(True)
    yr = torch.nn.functional.layer_norm(xr, (d,), gr, br, eps=1e-12)
    yr.backward(dy.double().cpu())
    ytol = dict(atol=1e-5, rtol=1e-5) if dt == torch.float32 else dict(atol=3e-2, rtol=1e-2)
    torch.testing.assert_close(y.double().cpu(), yr.detach(), **ytol)
    torch.testing.assert_close(dx.double().cpu(), dx0.double().cpu() + xr.grad, atol=2e-4, rtol=1e-4)
    torch.testing.assert_close(dparams[:d].double().cpu(), pg[:d].double().cpu() + gr.grad, atol=2e-3, rtol=1e-4)
    torch.testing.assert_close(dparams[d:].double().cpu(), pg[d:].double().cpu() + br.grad, atol=2e-3, rtol=1e-4)


@pytest.mark.parametrize("rows,cols,dt", [(7968, 512, torch.bfloat16), (1312, 2048, torch.float32),
                                          (50, 30, torch.bfloat16)])
def test_scale_dropout_colsum_matches_two_pass(rows, cols, dt):
    """Fused y = dropout(scale*x) + bias-gradient column sums == ea_scale_dropout then
    ea_colsum: identical y (same mask), column sums to f32 rounding (different partition)."""
    from espnet_amd import hip_ops as ops
    from espnet_amd._lib import lib
    lib.ea_set_rng_salt(None)  # a model built by an earlier test may have left its (freed) salt
    g = torch.Generator().manual_seed(rows)
    x = torch.randn(rows, cols, generator=g).cuda()
    y1 = torch.empty(rows, cols, dtype=dt, device="cuda")
    y2 = torch.empty_like(y1)
    c1 = torch.ones(cols, device="cuda")
    c2 = torch.ones(cols, device="cuda")
    w, wn = ops._ws(x.device)
    lib.ea_scale_dropout_colsum(rows, cols, x.data_ptr(), cols, y1.data_ptr(), ops.dt(y1), cols, 0.5, 0.1, 1234,
                                c1.data_ptr(), 1, w, wn, ops.stream())
    ops.scale_dropout(x, y2, scale=0.5, p=0.1, seed=1234)
    ops.colsum(y2, c2)
    torch.cuda.synchronize()
    assert torch.equal(y1, y2)
    drop = (y1 == 0).float().mean().item()
    assert 0.08 < drop < 0.12
    torch.testing.assert_close(c1, c2, atol=1e-3, rtol=1e-5)
    torch.testing.assert_close(c1.double().cpu(), 1 + y2.double().sum(0).cpu(), atol=1e-3, rtol=1e-5)


def test_grouped_reductions_match_per_call():
    """Deferred parameter-gradient reductions (ReduceQueue: grouped column sums + grouped
    ordered reductions, LayerNorm partials) equal the per-call ea_colsum / ea_layernorm_bwd
    results bit for bit, including strided inputs, f32/bf16 and accumulate."""
    from espnet_amd import hip_ops as ops
    g = torch.Generator().manual_seed(4)
    dev = "cuda"
    xs = [torch.randn(7968, 2048, generator=g).to(dev).to(torch.bfloat16),
          torch.randn(1312, 5000, generator=g).to(dev).to(torch.bfloat16),
          torch.randn(300, 3 * 64, generator=g).to(dev)[:, :64],   # strided f32 view
          torch.randn(33, 512, generator=g).to(dev)]
    outs0 = [torch.randn(x.shape[1], generator=g).to(dev) for x in xs]
    ref = [o.clone() for o in outs0]
    for x, o in zip(xs, ref):
        ops.colsum(x, o, accumulate=True)
    # LayerNorm: d=512 rows 7968, bf16 dy
    d, R = 512, 7968
    x = torch.randn(R, d, generator=g).to(dev)
    dy = torch.randn(R, d, generator=g).to(dev).to(torch.bfloat16)
    gamma = torch.randn(d, generator=g).to(dev)
    mean, rstd = x.mean(1), x.var(1, unbiased=False).add(1e-12).rsqrt()
    gb_ref = torch.randn(2 * d, generator=g).to(dev)
    gb_def = gb_ref.clone()
    dx_ref = torch.zeros(R, d, device=dev)
    dx_def = torch.zeros(R, d, device=dev)
    ops.layernorm_bwd(dy, x, gamma, mean, rstd, dx_ref, gb_ref[:d], gb_ref[d:], accumulate=True)
    outs = [o.clone() for o in outs0]
    with ops.deferred_wgrad():
        if ops.DEFER_REDUCE:
            for x_, o in zip(xs, outs):
                ops.colsum(x_, o, accumulate=True)
            ops.layernorm_bwd(dy, x, gamma, mean, rstd, dx_def, gb_def[:d], gb_def[d:], accumulate=True)
            assert len(ops.REDUCE_Q.colsums) == 4 and len(ops.REDUCE_Q.reduces) == 1
    torch.cuda.synchronize()
    if ops.DEFER_REDUCE:
        for o, r in zip(outs, ref):
            assert torch.equal(o, r)
        assert torch.equal(dx_def, dx_ref)
        assert torch.equal(gb_def, gb_ref)


@pytest.mark.parametrize("rows,d,ydt", [(7968, 512, torch.bfloat16), (1312, 1024, torch.bfloat16),
                                        (100, 80, torch.bfloat16), (257, 256, torch.float32)])
@pytest.mark.parametrize("partials", [False, True])
@pytest.mark.parametrize("dyt", [torch.bfloat16, torch.float32])
def test_layernorm_bwd_drop_matches_two_pass(rows, d, ydt, partials, dyt):
    """ea_layernorm_bwd_drop / _partials_drop (dx, the next site's y = dropout(scale*dx) and its
    column sums) vs ea_layernorm_bwd / _partials then ea_scale_dropout, in-kernel (bf16 y,
    vector rows) and pass fallback: y bit-identical to the dropout of the launch's own dx,
    column sums = f64 sums of the stored y."""
    import ctypes
    from espnet_amd import hip_ops as ops
    from espnet_amd._lib import lib
    lib.ea_set_rng_salt(None)
    g = torch.Generator().manual_seed(rows * d)
    x = (torch.randn(rows, d, generator=g) * 2 + 1).cuda()
    gamma = (torch.rand(d, generator=g) + 0.5).cuda()
    beta = torch.randn(d, generator=g).cuda()
    dy = torch.randn(rows, d, generator=g).to(dyt).cuda()
    yln = torch.empty(rows, d, dtype=torch.bfloat16, device="cuda")
    mu = torch.empty(rows, device="cuda")
    rs = torch.empty(rows, device="cuda")
    ops.layernorm_fwd(x, gamma, beta, yln, mu, rs)
    dx0 = torch.randn(rows, d, generator=g).cuda()
    ycol0 = torch.randn(d, generator=g).cuda()
    res = []
    for fused in (False, True):
        dx = dx0.clone()
        y = torch.empty(rows, d, dtype=ydt, device="cuda")
        par = torch.zeros(2 * d, device="cuda")
        ycol = ycol0.clone()
        if partials:
            part = torch.empty(max((rows + 15) // 16, 128) * 3 * d, device="cuda")
            npart, yparts = ctypes.c_int(0), ctypes.c_int(0)
            args = (rows, d, dy.data_ptr(), ops.dt(dy), d, x.data_ptr(), d, gamma.data_ptr(), mu.data_ptr(),
                    rs.data_ptr(), dx.data_ptr(), d, 1, part.data_ptr(), part.numel(), ctypes.addressof(npart))
            if fused:
                lib.ea_layernorm_bwd_partials_drop(*args, y.data_ptr(), ops.dt(y), d, 0.5, 0.1, 99, ycol.data_ptr(),
                                                   ctypes.addressof(yparts), ops.stream())
            else:
                lib.ea_layernorm_bwd_partials(*args, ops.stream())
            n = npart.value
            ops.reduce_rows(part, n, 2 * d, 2 * d, par)
            if yparts.value:
                ops.reduce_rows(part[n * 2 * d:], n, d, d, ycol)
            assert yparts.value == int(fused and ydt == torch.bfloat16 and d % 8 == 0)
        else:
            ops.layernorm_bwd(dy, x, gamma, mu, rs, dx, par[:d], par[d:], accumulate=True,
                              drop=(y, 0.5, 0.1, 99, ycol) if fused else None)
        if not fused:
            ops.scale_dropout(dx, y, scale=0.5, p=0.1, seed=99)
        torch.cuda.synchronize()
        res.append((dx, y, par, ycol))
    (dx1, y1, p1, _), (dx2, y2, p2, c2) = res
    # y is exactly the site's dropout of the dx this launch wrote; dx and the parameter sums
    # match the plain kernel to f32 rounding (the compiler may contract the variants' FMAs
    # differently)
    y3 = torch.empty_like(y2)
    ops.scale_dropout(dx2, y3, scale=0.5, p=0.1, seed=99)
    torch.cuda.synchronize()
    assert torch.equal(y2, y3)
    torch.testing.assert_close(dx2, dx1, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(p2, p1, atol=1e-4, rtol=1e-5)
    torch.testing.assert_close(y2.float(), y1.float(), atol=1e-2, rtol=1e-2)
    torch.testing.assert_close(c2.double().cpu(), ycol0.double().cpu() + y2.double().sum(0).cpu(), atol=2e-3,
                               rtol=1e-5)
    assert 0.08 < (y2 == 0).float().mean().item() < 0.12
