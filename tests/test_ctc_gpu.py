"""CTC loss C-ABI (ea_ctc_loss_fwd / ea_ctc_loss_bwd: lse + alpha/beta lattice + fused
gradient) against the reference's CTC golden (tests/golden/ctc_op.npz: torch CTCLoss
reduction=none, zero_infinity=True, ragged and infeasible utterances) and, at C3-like sizes,
against torch's CPU CTCLoss on the same logits."""
import numpy as np
import pytest
import torch

from goldens import load

pytestmark = pytest.mark.gpu


def run_ctc(logits_btv, ilens, ys, ylens):
    from espnet_amd._lib import lib
    from espnet_amd import hip_ops as ops
    B, T, V = logits_btv.shape
    Lmax = ys.shape[1]
    S = 2 * Lmax + 1
    dev = torch.device("cuda")
    x = logits_btv.contiguous().to(dev)
    il, yy, yl = ilens.to(dev), ys.to(dev).contiguous(), ylens.to(dev)
    lse = torch.empty(B * T, device=dev)
    alpha = torch.empty(B * T * S, dtype=torch.float64, device=dev)
    beta = torch.empty_like(alpha)
    nll = torch.empty(B, dtype=torch.float64, device=dev)
    loss_utt = torch.empty(B, device=dev)
    loss = torch.empty((), device=dev)
    lib.ea_ctc_loss_fwd(B, T, V, x.data_ptr(), V, il.data_ptr(), yy.data_ptr(), yy.stride(0), yl.data_ptr(), Lmax,
                        lse.data_ptr(), alpha.data_ptr(), beta.data_ptr(), nll.data_ptr(), loss_utt.data_ptr(),
                        loss.data_ptr(), ops.stream())
    gs = torch.ones(1, device=dev)
    grad = torch.empty(B * T, V, device=dev)
    lib.ea_ctc_loss_bwd(B, T, V, x.data_ptr(), V, il.data_ptr(), yy.data_ptr(), yy.stride(0), yl.data_ptr(), Lmax,
                        lse.data_ptr(), alpha.data_ptr(), beta.data_ptr(), nll.data_ptr(), gs.data_ptr(), 1.0 / B,
                        grad.data_ptr(), 0, V, ops.stream())
    torch.cuda.synchronize()
    return loss_utt.cpu(), loss.cpu(), grad.view(B, T, V).cpu()


def test_ctc_matches_reference_golden():
    _, d = load("ctc_op")
    logits = torch.from_numpy(d["logits"]).transpose(0, 1)  # (B, T, V)
    B = logits.shape[0]
    ol = d["olens"]
    ys = np.full((B, max(ol.max(), 1)), -1, dtype=np.int64)
    off = 0
    for b, l in enumerate(ol):
        ys[b, :l] = d["target"][off:off + l]
        off += l
    lu, loss, grad = run_ctc(logits, torch.from_numpy(d["ilens"]), torch.from_numpy(ys), torch.from_numpy(ol))
    np.testing.assert_allclose(lu.numpy(), d["loss_utt"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(loss.item(), d["loss"], rtol=1e-6, atol=1e-5)
    # the gradient kernel's softmax uses the fast f32 exp: ~1e-6 absolute at |g| ~ 0.2
    np.testing.assert_allclose(grad.numpy(), d["grad_logits"].transpose(1, 0, 2), atol=5e-6, rtol=1e-4)


@pytest.mark.parametrize("B,T,V,L", [(32, 249, 5000, 40), (4, 499, 300, 80), (3, 70, 50, 130)])
def test_ctc_long_sequences_vs_torch(B, T, V, L):
    """C3 sizes (32 x 249 frames, 40 labels), C5 sizes (499 frames, 80 labels), and a label
    sequence longer than the two-workgroup lattice's 256 states (one-workgroup fallback)."""
    g = torch.Generator().manual_seed(B * T + L)
    logits = torch.randn(B, T, V, generator=g)
    ilens = torch.randint(max(T // 2, 2 * L + 2) if 2 * L + 2 <= T else T // 2, T + 1, (B,), generator=g)
    ilens[0] = T
    ylens = torch.randint(1, L + 1, (B,), generator=g)
    ylens[0] = L
    ys = torch.full((B, L), -1, dtype=torch.long)
    for b in range(B):
        ys[b, :ylens[b]] = torch.randint(1, V, (int(ylens[b]),), generator=g)
    lu, loss, grad = run_ctc(logits, ilens, ys, ylens)
    # reference in f64: torch's f32 CPU lattice drifts (its per-frame occupancies sum to
    # 1 - 6e-4 at T=499), which log_softmax backward turns into a uniform gradient scale
    x = logits.double().requires_grad_(True)
    lp = torch.log_softmax(x, dim=-1).transpose(0, 1)
    tgt = torch.cat([ys[b, :ylens[b]] for b in range(B)])
    ref = torch.nn.CTCLoss(reduction="none", zero_infinity=True)(lp, tgt, ilens, ylens)
    (ref.sum() / B).backward()
    np.testing.assert_allclose(lu.numpy(), ref.detach().numpy(), rtol=2e-6, atol=1e-4)
    np.testing.assert_allclose(grad.numpy(), x.grad.numpy(), atol=2e-6, rtol=1e-4)


def test_ctc_prefix_kernel_matches_numpy_restatement():
    """ea_ctc_prefix_init / ea_ctc_prefix_score against the numpy CTCPrefixScore restatement
    (oracle, pinned to the reference beam-search goldens): initial state, prefix scores and
    next forward variables for prefixes of length 0..3, repeated labels, <eos> and blank
    among the candidates."""
    import numpy as np
    import torch
    from espnet_amd._lib import lib
    from espnet_amd import hip_ops as ops
    from oracle.asr_oracle import OracleCTCPrefixScore
    g = torch.Generator().manual_seed(5)
    T, V, eos = 37, 11, 10
    logits = torch.randn(T, V, generator=g) * 2
    logp_ref = torch.log_softmax(logits, -1).numpy()
    impl = OracleCTCPrefixScore(logp_ref, 0, eos)
    lg = logits.cuda()
    logp = torch.empty(T, V, device="cuda")
    r0 = torch.empty(T, 2, device="cuda")
    lib.ea_ctc_prefix_init(T, V, lg.data_ptr(), V, 0, logp.data_ptr(), r0.data_ptr(), ops.stream())
    np.testing.assert_allclose(logp.cpu().numpy(), logp_ref, atol=2e-6)
    np.testing.assert_allclose(r0.cpu().numpy(), impl.initial_state(), rtol=1e-5, atol=1e-5)
    cs = np.array([0, 3, 5, 7, eos], dtype=np.int64)
    for y in ([eos], [eos, 3], [eos, 3, 5], [eos, 3, 5, 5]):
        # previous state: the restatement's own recursion along y
        r_prev = impl.initial_state()
        for k in range(1, len(y)):
            _, st = impl(np.array(y[:k]), np.array([y[k]]), r_prev)
            r_prev = st[0]
        psi_ref, r_ref = impl(np.array(y), cs, r_prev)
        rp = torch.from_numpy(np.ascontiguousarray(r_prev)).cuda()
        meta = torch.tensor([len(y) - 1, y[-1]] + cs.tolist(), dtype=torch.int32, device="cuda")
        ptrs = torch.tensor([rp.data_ptr()], dtype=torch.int64, device="cuda")
        psi = torch.empty(len(cs), device="cuda")
        rn = torch.empty(len(cs), T, 2, device="cuda")
        lib.ea_ctc_prefix_score(T, V, 0, eos, 1, len(cs), logp.data_ptr(), ptrs.data_ptr(), meta.data_ptr(),
                                psi.data_ptr(), rn.data_ptr(), ops.stream())
        torch.cuda.synchronize()
        np.testing.assert_allclose(psi.cpu().numpy(), psi_ref, rtol=1e-5, atol=1e-4)
        ol = len(y) - 1
        lo = max(ol, 1) - 1  # rows below the start are never read by the reference
        np.testing.assert_allclose(rn.cpu().numpy()[:, lo:], r_ref[:, lo:], rtol=1e-5, atol=1e-4)


def test_ctc_softmax_log_softmax_api():
    """CTC.softmax / CTC.log_softmax / CTC.argmax (espnet2/asr/ctc.py:99-127) on the HIP
    path against torch fp32 of the same ctc_lo logits."""
    from goldens import load, section
    from test_model_build import build
    cfg, d = load("tiny_hybrid")
    torch.manual_seed(0)
    m = build(cfg)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in section(d, "w").items()})
    m.prepare("cuda:0", amp=False)
    hs = torch.from_numpy(d["out.encoder_out"]).cuda()
    lg = m.ctc.logits(hs).double().cpu()
    sm = m.ctc.softmax(hs).double().cpu()
    lsm = m.ctc.log_softmax(hs).double().cpu()
    torch.testing.assert_close(sm, torch.softmax(lg, dim=2), atol=1e-6, rtol=1e-5)
    torch.testing.assert_close(lsm, torch.log_softmax(lg, dim=2), atol=1e-5, rtol=1e-6)
    assert torch.equal(m.ctc.argmax(hs).cpu(), lg.argmax(2))
