"""CPU restatement of the validation error rates — ORACLE, TEST INFRASTRUCTURE ONLY.

Only tests/ may import this module, as the checker. Restates
espnet/nets/e2e_asr_common.py:100-256 (ErrorCalculator: convert_to_char, calculate_cer,
calculate_wer, calculate_cer_ctc). The reference's edit distance comes from the third-party
`editdistance` package (PyPI, unpinned in setup.py; absent here); its published algorithm,
unit-cost Levenshtein over sequence elements, is restated below as the full (n+1)x(m+1)
numpy table, so it shares no code with the product's two-row version.

Pinning: the edit distance against editdistance's published known answers and hand-derived
cases (tests/test_error_calculator.py); the string handling around it is PARITY UNPINNED
against the reference itself (ErrorCalculator cannot run here without editdistance).
"""
from __future__ import annotations

import numpy as np


def levenshtein(a, b) -> int:
    a, b = list(a), list(b)
    D = np.zeros((len(a) + 1, len(b) + 1), dtype=np.int64)
    D[:, 0] = np.arange(len(a) + 1)
    D[0, :] = np.arange(len(b) + 1)
    for i in range(1, len(a) + 1):
        for j in range(1, len(b) + 1):
            D[i, j] = min(D[i - 1, j] + 1, D[i, j - 1] + 1, D[i - 1, j - 1] + (a[i - 1] != b[j - 1]))
    return int(D[-1, -1])


def _strip(ids, skip):
    return [int(i) for i in ids if int(i) not in skip]


def oracle_cer_ctc(ys_hat, ys_pad, char_list, blank="<blank>", space="<space>"):
    """e2e_asr_common.py:160-193."""
    skip = {-1}
    if blank in char_list:
        skip.add(char_list.index(blank))
    if space in char_list:
        skip.add(char_list.index(space))
    eds = lens = 0
    for y_hat, y_true in zip(np.asarray(ys_hat), np.asarray(ys_pad)):
        collapsed = [int(v) for k, v in enumerate(y_hat) if k == 0 or y_hat[k - 1] != v]
        hyp = "".join(char_list[i] for i in _strip(collapsed, skip))
        ref = "".join(char_list[i] for i in _strip(y_true, skip))
        if len(ref) > 0:
            eds += levenshtein(hyp, ref)
            lens += len(ref)
    return eds / lens if lens else None


def oracle_cer_wer(ys_hat, ys_pad, char_list, blank="<blank>", space="<space>"):
    """e2e_asr_common.py:195-256: hypothesis cut at the reference's first -1, space token ->
    ' ', blank token text removed; CER over space-free characters, WER over words."""
    ce = cl = we = wl = 0
    for y_hat, y_true in zip(np.asarray(ys_hat), np.asarray(ys_pad)):
        pad = np.nonzero(y_true == -1)[0]
        ymax = int(pad[0]) if len(pad) else len(y_true)
        hyp = "".join(char_list[int(i)] for i in y_hat[:ymax]).replace(space, " ").replace(blank, "")
        ref = "".join(char_list[int(i)] for i in y_true if i != -1).replace(space, " ")
        ce += levenshtein(hyp.replace(" ", ""), ref.replace(" ", ""))
        cl += len(ref.replace(" ", ""))
        we += levenshtein(hyp.split(), ref.split())
        wl += len(ref.split())
    return ce / cl, we / wl
