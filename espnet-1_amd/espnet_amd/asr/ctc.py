"""CTC — drop-in for espnet2/asr/ctc.py:6-127 (builtin ctc_type).  forward returns the
batch-summed loss / B like the reference (reduce=True); argmax gives the greedy CTC
alignment (bit-exact index requirement)."""
from __future__ import annotations

import torch
from torch import nn

from ..layers.common import Bound, empty, lib, ops
from ..layers.losses import CTCFn


class CTC(nn.Module):
    def __init__(self, odim: int, encoder_output_size: int, dropout_rate: float = 0.0,
                 ctc_type: str = "builtin", reduce: bool = True, ignore_nan_grad: bool = None,
                 zero_infinity: bool = True):
        super().__init__()
        eprojs = encoder_output_size
        self.dropout_rate = dropout_rate
        self.ctc_lo = nn.Linear(eprojs, odim)
        self.ctc_type = ctc_type
        if ignore_nan_grad is not None:
            zero_infinity = ignore_nan_grad
        if ctc_type not in ("builtin", "gtnctc"):
            raise ValueError(f'ctc_type must be "builtin" or "gtnctc": {ctc_type}')
        if ctc_type != "builtin" or not zero_infinity or not reduce:
            raise NotImplementedError("espnet_amd CTC implements ctc_type=builtin, zero_infinity=True, "
                                      "reduce=True (the training path)")
        self.reduce = reduce
        self.zero_infinity = zero_infinity
        self._b = None
        self._seed = 0
        self._overlap = False

    def bind(self, arena, prefix, cd):
        self._b = Bound(arena, prefix, cd)

    def forward(self, hs_pad, hlens, ys_pad, ys_lens, seed: int = 0, overlap: bool = False):
        """ctc.py:72-97.  ys_pad (B, Lmax) padded with -1; returns sum_b loss_b / B.
        overlap=True: the lattice runs on the auxiliary stream (hip_ops.aux) and the caller
        must hip_ops.join_aux() before using the loss (ESPnetASRModel.forward does)."""
        self._seed = seed
        self._overlap = overlap
        return CTCFn.apply(hs_pad.contiguous(), hlens, ys_pad.contiguous(), ys_lens, self,
                           int(ys_pad.shape[1]))

    @torch.no_grad()
    def logits(self, hs_pad):
        b = self._b
        B, T, d = hs_pad.shape
        h = ops.cast(hs_pad.reshape(B * T, d).contiguous(), b.cd)
        out = empty(B * T, self.ctc_lo.out_features, device=hs_pad.device)
        ops.linear(h, b.w("ctc_lo.weight"), out, epi=ops.make_epi(bias=b.f("ctc_lo.bias")))
        return out.view(B, T, -1)

    @torch.no_grad()
    def _softmax(self, hs_pad, log):
        lg = self.logits(hs_pad)
        B, T, V = lg.shape
        out = torch.empty_like(lg)
        lib.ea_softmax_rows(B * T, V, lg.data_ptr(), V, out.data_ptr(), int(log), ops.stream())
        return out

    def softmax(self, hs_pad):
        """ctc.py:99-107: softmax(ctc_lo(hs_pad), dim=2) -> (B, T, V).  An inference helper
        here (no autograd; the interCTC conditioning that differentiates it is not built)."""
        return self._softmax(hs_pad, False)

    def log_softmax(self, hs_pad):
        """ctc.py:109-117: log_softmax(ctc_lo(hs_pad), dim=2) -> (B, T, V) (decoding's CTC
        prefix scorer input); no autograd."""
        return self._softmax(hs_pad, True)

    @torch.no_grad()
    def argmax(self, hs_pad):
        """ctc.py:119-127: argmax over the vocabulary of ctc_lo(hs_pad) -> (B, T) int64."""
        lg = self.logits(hs_pad)
        B, T, V = lg.shape
        out = torch.empty(B, T, dtype=torch.long, device=hs_pad.device)
        lib.ea_argmax_rows(B * T, V, lg.data_ptr(), V, out.data_ptr(), ops.stream())
        return out
