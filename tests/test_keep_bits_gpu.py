"""The Conformer FFN's activation-dropout keep bits (layers/conformer.py KEEP_BITS: the w_1
forward epilogue writes its decisions, the w_2 input-gradient epilogue reads them) give the
same training step, bit for bit, as re-hashing the dropout stream in the backward — bf16 AMP,
dropout 0.1, two steps of the tiny hybrid model."""
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)


def _steps(keep_bits):
    from test_dp_capture_gpu import _batches, _setup
    from espnet_amd.layers import conformer as C
    from espnet_amd.train.trainer import Trainer
    saved = C.KEEP_BITS
    C.KEEP_BITS = keep_bits
    try:
        d, m, opt, sched = _setup(amp=True, dropout=0.1)
        losses = [float(Trainer.train_one_step(m, b, opt, sched, grad_clip=5.0)[0]) for b in _batches(d, 2)]
        torch.cuda.synchronize()
        return losses, m.arena.data.cpu().clone()
    finally:
        C.KEEP_BITS = saved


def test_ffn_keep_bits_step_bit_identical():
    l0, w0 = _steps(False)
    l1, w1 = _steps(True)
    assert l0 == l1
    assert torch.equal(w0, w1)
