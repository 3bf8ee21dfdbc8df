"""Validation CER/WER (espnet/nets/e2e_asr_common.py:100-250, ErrorCalculator).

ESPnetASRModel builds one when report_cer or report_wer (espnet2/asr/espnet_model.py:164-167)
and calls it in eval mode only: on the attention decoder's argmax (espnet_model.py:551-557,
`cer`/`wer`) and on the CTC frame argmax (espnet_model.py:571-575, `cer_ctc`). The argmaxes
run on the device (ea_argmax_rows); what reaches this class is two small (B, L) / (B, T')
index tensors, so the string work stays on the host like the reference's.

The reference scores with the third-party `editdistance` package (not installed here); its
published algorithm is the unit-cost Levenshtein distance over sequence elements (characters
of a str, items of a list), restated in `edit_distance` below.
"""
from __future__ import annotations

from itertools import groupby
from typing import List, Optional, Sequence

import numpy as np


def edit_distance(hyp: Sequence, ref: Sequence) -> int:
    """Unit-cost Levenshtein distance (editdistance.eval). One numpy pass per hypothesis
    element: the substitution/deletion terms are elementwise over the previous row, and the
    insertion chain cur[j] = min_k<=j (t[k] + j - k) is j + a cumulative minimum of t[k] - k,
    so a row costs a few vector ops instead of a Python loop over the reference."""
    if len(hyp) < len(ref):
        hyp, ref = ref, hyp
    if len(ref) == 0:
        return len(hyp)
    ids: dict = {}
    h = np.fromiter((ids.setdefault(x, len(ids)) for x in hyp), dtype=np.int64, count=len(hyp))
    r = np.fromiter((ids.setdefault(x, len(ids)) for x in ref), dtype=np.int64, count=len(ref))
    ramp = np.arange(len(r) + 1, dtype=np.int64)
    prev = ramp.copy()
    t = np.empty_like(prev)
    for i, x in enumerate(h, 1):
        t[0] = i
        np.minimum(prev[1:] + 1, prev[:-1] + (r != x), out=t[1:])
        prev = np.minimum.accumulate(t - ramp) + ramp
    return int(prev[-1])


def _rows(t) -> List[List[int]]:
    return [[int(v) for v in row] for row in (t.tolist() if hasattr(t, "tolist") else t)]


class ErrorCalculator:
    """Same constructor and __call__ contract as the reference: __call__(ys_hat, ys_pad) ->
    (cer, wer) with None for the disabled ones; __call__(..., is_ctc=True) -> cer_ctc."""

    def __init__(self, char_list, sym_space, sym_blank, report_cer=False, report_wer=False):
        self.report_cer = report_cer
        self.report_wer = report_wer
        self.char_list = list(char_list)
        self.space = sym_space
        self.blank = sym_blank
        self.idx_blank = self.char_list.index(sym_blank) if sym_blank in self.char_list else None
        self.idx_space = self.char_list.index(sym_space) if sym_space in self.char_list else None

    def __call__(self, ys_hat, ys_pad, is_ctc: bool = False):
        if is_ctc:
            return self.calculate_cer_ctc(ys_hat, ys_pad)
        if not self.report_cer and not self.report_wer:
            return None, None
        seqs_hat, seqs_true = self.convert_to_char(ys_hat, ys_pad)
        cer = self.calculate_cer(seqs_hat, seqs_true) if self.report_cer else None
        wer = self.calculate_wer(seqs_hat, seqs_true) if self.report_wer else None
        return cer, wer

    def _chars(self, ids) -> str:
        skip = (-1, self.idx_blank, self.idx_space)
        return "".join(self.char_list[i] for i in ids if i not in skip)

    def calculate_cer_ctc(self, ys_hat, ys_pad) -> Optional[float]:
        """e2e_asr_common.py:160-193: collapse repeats over every frame of the padded
        argmax, drop -1 / blank / space, character edit distance over the joined tokens;
        utterances with an empty reference are skipped."""
        errs = refs = 0
        for y_hat, y_true in zip(_rows(ys_hat), _rows(ys_pad)):
            hyp = self._chars([k for k, _ in groupby(y_hat)])
            ref = self._chars(y_true)
            if ref:
                errs += edit_distance(hyp, ref)
                refs += len(ref)
        return float(errs) / refs if refs else None

    def convert_to_char(self, ys_hat, ys_pad):
        """e2e_asr_common.py:195-220: the hypothesis is cut at the reference's first -1."""
        seqs_hat, seqs_true = [], []
        for y_hat, y_true in zip(_rows(ys_hat), _rows(ys_pad)):
            ymax = y_true.index(-1) if -1 in y_true else len(y_true)
            hyp = "".join(self.char_list[i] for i in y_hat[:ymax]).replace(self.space, " ")
            hyp = hyp.replace(self.blank, "")
            ref = "".join(self.char_list[i] for i in y_true if i != -1).replace(self.space, " ")
            seqs_hat.append(hyp)
            seqs_true.append(ref)
        return seqs_hat, seqs_true

    def calculate_cer(self, seqs_hat, seqs_true) -> float:
        """e2e_asr_common.py:222-238 (spaces removed, character distance)."""
        errs = sum(edit_distance(h.replace(" ", ""), r.replace(" ", "")) for h, r in zip(seqs_hat, seqs_true))
        return float(errs) / sum(len(r.replace(" ", "")) for r in seqs_true)

    def calculate_wer(self, seqs_hat, seqs_true) -> float:
        """e2e_asr_common.py:240-256 (whitespace-split words)."""
        errs = sum(edit_distance(h.split(), r.split()) for h, r in zip(seqs_hat, seqs_true))
        return float(errs) / sum(len(r.split()) for r in seqs_true)
