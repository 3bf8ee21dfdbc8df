"""Adam update kernel (ea_adam_step: torch.optim.Adam arithmetic, grad-clip coefficient,
bf16 shadow) against an f32 torch restatement of the same element formula (odd n, aligned
and misaligned views)."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,off", [(1_000_003, 0), (4096, 0), (777, 1)])
def test_adam_step_matches_restatement(n, off):
    from espnet_amd import hip_ops as ops
    from espnet_amd._lib import lib
    g_ = torch.Generator().manual_seed(n)
    buf = lambda s=1.0: (torch.randn(n + 4, generator=g_) * s).cuda()  # noqa: E731
    p, g, m, v = buf(), buf(0.1), buf(0.01), buf(0.001).abs()
    p16 = torch.empty(n + 4, dtype=torch.bfloat16, device="cuda")
    norm = torch.tensor([7.5], device="cuda")
    lr, b1, b2, eps, wd, step, max_norm = 1e-3, 0.9, 0.98, 1e-9, 1e-6, 3, 5.0
    ref = [t[off:off + n].clone() for t in (p, g, m, v)]
    sl = lambda t: t[off:off + n]  # noqa: E731
    lib.ea_adam_step(n, sl(p).data_ptr(), sl(g).data_ptr(), sl(m).data_ptr(), sl(v).data_ptr(),
                     sl(p16).data_ptr(), lr, b1, b2, eps, wd, step, norm.data_ptr(), max_norm, ops.stream())
    torch.cuda.synchronize()
    rp, rg, rm, rv = ref
    coef = min(max_norm / (7.5 + 1e-6), 1.0)
    gg = rg * coef + wd * rp
    rm = rm + (1 - b1) * (gg - rm)
    rv = rv * b2 + (1 - b2) * gg * gg
    denom = rv.sqrt() / math.sqrt(1 - b2 ** step) + eps
    rp = rp - (lr / (1 - b1 ** step)) * (rm / denom)
    # a few ulps of each state's scale (the kernel may contract the lerp / moment updates
    # into FMAs; torch rounds every op)
    torch.testing.assert_close(sl(m), rm, rtol=1e-6, atol=3e-8)
    torch.testing.assert_close(sl(v), rv, rtol=1e-6, atol=3e-9)
    torch.testing.assert_close(sl(p), rp, rtol=1e-6, atol=3e-7)
    assert torch.equal(sl(p16), sl(p).to(torch.bfloat16))
