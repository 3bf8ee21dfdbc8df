"""Row/utterance reductions of the step's input and loss ends through the C-ABI:
utterance MVN (ea_utterance_mvn2, chunked two-pass; ea_utterance_mvn, one block per
utterance) against the oracle's utterance_mvn in f64, and the label-smoothing loss forward
(ea_lsm_loss_fwd: row lse, KL vs the smoothed target, ignore_id rows, th_accuracy counts)
against an f64 torch restatement of label_smoothing_loss.py:41-63 / nets_utils.py:304-324,
on 16-B aligned rows (float4 path) and odd-stride rows (scalar path)."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,T,F", [(32, 1598, 80), (3, 31, 80), (5, 97, 256), (2, 1, 7), (4, 64, 83)])
def test_utterance_mvn_chunked_matches_oracle(B, T, F):
    from espnet_amd._lib import lib
    from espnet_amd import hip_ops as ops
    from oracle.asr_oracle import utterance_mvn
    g = torch.Generator().manual_seed(B * T + F)
    x = torch.randn(B, T, F, generator=g) * 4 + 2
    lens = torch.randint(1, T + 1, (B,), generator=g)
    lens[0] = T
    xd, ld = x.cuda(), lens.cuda()
    n = ctypes.c_long(0)
    assert lib.ea_utterance_mvn_ws_bytes(B, T, F, ctypes.addressof(n)) == 0
    ws = torch.full((max(n.value, 8),), 0xFF, dtype=torch.uint8, device="cuda")  # garbage: fully rewritten
    y2 = torch.empty_like(xd)
    y1 = torch.empty_like(xd)
    assert lib.ea_utterance_mvn2(B, T, F, xd.data_ptr(), ld.data_ptr(), y2.data_ptr(), ws.data_ptr(), ws.numel(),
                                 ops.stream()) == 0
    assert lib.ea_utterance_mvn(B, T, F, xd.data_ptr(), ld.data_ptr(), y1.data_ptr(), ops.stream()) == 0
    torch.cuda.synchronize()
    ref = utterance_mvn(x.double(), lens).numpy()
    np.testing.assert_allclose(y2.cpu().numpy(), ref, rtol=1e-6, atol=2e-6)
    np.testing.assert_allclose(y2.cpu().numpy(), y1.cpu().numpy(), rtol=0, atol=2e-6)
    # too small a workspace is refused (EA_ERR_BAD_ARG, raised by the binding)
    from espnet_amd._lib import HipError
    with pytest.raises(HipError, match="bad argument"):
        lib.ea_utterance_mvn2(B, T, F, xd.data_ptr(), ld.data_ptr(), y2.data_ptr(), ws.data_ptr(), n.value - 8,
                              ops.stream())


@pytest.mark.parametrize("rows,V,ldx", [(1312, 5000, 5000), (77, 50, 50), (64, 301, 303), (9, 4, 4)])
def test_lsm_loss_fwd_matches_f64_restatement(rows, V, ldx):
    from espnet_amd._lib import lib
    from espnet_amd import hip_ops as ops
    g = torch.Generator().manual_seed(rows + V)
    x = torch.randn(rows, ldx, generator=g) * 3
    x[3 % rows, :V] = 1.0  # all-equal row: argmax is the first index
    tgt = torch.randint(0, V, (rows,), generator=g)
    tgt[::7] = -1  # ignore_id
    tgt[3 % rows] = 0
    sm, ign = 0.1, -1
    xd, td = x.cuda(), tgt.cuda()
    lse = torch.empty(rows, device="cuda")
    loss_row = torch.empty(rows, dtype=torch.float64, device="cuda")
    stat = torch.empty(2, dtype=torch.int32, device="cuda")
    loss, acc, inv = (torch.empty(1, device="cuda") for _ in range(3))
    assert lib.ea_lsm_loss_fwd(rows, V, xd.data_ptr(), ldx, td.data_ptr(), sm, ign, 1, 1.0, lse.data_ptr(),
                               loss_row.data_ptr(), stat.data_ptr(), loss.data_ptr(), acc.data_ptr(),
                               inv.data_ptr(), ops.stream()) == 0
    torch.cuda.synchronize()
    xv = x[:, :V].double()
    lse_ref = torch.logsumexp(xv, -1)
    valid = tgt != ign
    t0 = tgt.masked_fill(~valid, 0)
    q = torch.full((rows, V), sm / (V - 1), dtype=torch.float64)
    q.scatter_(1, t0[:, None], 1 - sm)
    kl = (q * (q.log() - (xv - lse_ref[:, None]))).sum(-1).masked_fill(~valid, 0)
    np.testing.assert_allclose(lse.cpu().numpy(), lse_ref.numpy(), rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(loss_row.cpu().numpy(), kl.numpy(), rtol=1e-6, atol=1e-6)
    am = xv.argmax(-1)
    assert stat.cpu().tolist() == [int(((am == tgt) & valid).sum()), int(valid.sum())]
    np.testing.assert_allclose(loss.item(), kl.sum().item() / int(valid.sum()), rtol=1e-6)
