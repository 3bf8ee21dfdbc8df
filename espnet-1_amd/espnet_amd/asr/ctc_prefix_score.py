"""Vectorised CTC prefix scoring — drop-in for espnet/nets/ctc_prefix_score.py:11-270
(CTCPrefixScoreTH, the batch scorer that espnet/nets/scorers/ctc.py:87-126 hands to
BatchBeamSearch).

Same constructor (x: (B, T, O) label log-posteriors, xlens, blank, eos, margin), the same
call (prefixes y of B * n_hyps hypotheses, previous state, optional pre-beam scoring_ids)
returning (local scores (B * n_hyps, O), state), and index_select_state(state, best_ids) with
best_ids in each utterance's (n_hyps * O) space.  Scores follow the reference: log psi of
every scored label minus the hypothesis's previous prefix score, logzero (-1e10) for labels
outside scoring_ids and for blank, the full-sequence probability for <eos>.

MI355X layout: the posteriors stay in HBM and every (hypothesis, candidate) pair of an
utterance is one thread of the CTC prefix kernel (csrc/ctc_prefix.hip, one launch per
utterance and step), walking the utterance's own frames only — the reference's padded frames
(logzero labels, log 1 blank) contribute nothing above f32 rounding, so they are not
visited.  A hypothesis's state is its (T_b, 2) forward variables in HBM.  Attention-windowed
scoring (margin > 0) and streaming extension (extend_prob / extend_state) are outside the
recipes' decoding and raise NotImplementedError.
"""
from __future__ import annotations

from typing import List

import torch

from .. import hip_ops as ops
from .._lib import lib

LOGZERO = -10000000000.0


class CTCPrefixScoreTH:
    def __init__(self, x: torch.Tensor, xlens, blank: int, eos: int, margin: int = 0):
        if margin > 0:
            raise NotImplementedError("CTCPrefixScoreTH: attention-windowed scoring (margin > 0)")
        if x.device.type != "cuda":
            raise RuntimeError("CTCPrefixScoreTH runs on the HIP device (x must be a device tensor)")
        self.logzero = LOGZERO
        self.blank, self.eos = int(blank), int(eos)
        self.batch, self.input_length, self.odim = (int(v) for v in x.shape)
        self.dtype, self.device = x.dtype, x.device
        self.xlens = [int(v) for v in xlens]
        # the reference pads the caller's tensor in place (ctc_prefix_score.py:45-50)
        for i, l in enumerate(self.xlens):
            if l < self.input_length:
                x[i, l:, :] = self.logzero
                x[i, l:, self.blank] = 0
        self.logp = [x[b, :l].float().contiguous() for b, l in enumerate(self.xlens)]
        self.r0 = []
        for lp in self.logp:  # initial state: (logzero, cumulative blank log-probability)
            r = torch.full((lp.shape[0], 2), self.logzero, dtype=torch.float32, device=self.device)
            r[:, 1] = torch.cumsum(lp[:, self.blank], 0)
            self.r0.append(r)
        self.scoring_num = 0

    def __call__(self, y: List[torch.Tensor], state, scoring_ids=None, att_w=None):
        n_bh = len(y)
        n_hyps = n_bh // self.batch
        out_len = len(y[0]) - 1
        last = [int(yy[-1]) for yy in y]
        if state is None:
            r_prev = [self.r0[i // n_hyps] for i in range(n_bh)]
            s_prev = torch.zeros(n_bh, 1, device=self.device)
        else:
            r_prev, s_prev = state[0], state[1]
        if scoring_ids is not None:
            cand = scoring_ids.to(torch.int64).cpu()
            self.scoring_num = int(cand.shape[-1])
        else:
            cand = torch.arange(self.odim, dtype=torch.int64).repeat(n_bh, 1)
            self.scoring_num = 0
        # <eos> always scored (the reference sets it for every hypothesis, :178-179); the
        # state lookup below sees only the scored columns, as the reference's scoring_idmap
        nsc = int(cand.shape[1])
        has_eos = (cand == self.eos).any(dim=1)
        if not bool(has_eos.all()):
            cand = torch.cat([cand, torch.full((n_bh, 1), self.eos, dtype=torch.int64)], dim=1)
        nc = int(cand.shape[1])
        log_psi = torch.full((n_bh, self.odim), self.logzero, dtype=torch.float32, device=self.device)
        r_new = []
        for b in range(self.batch):
            hs = range(b * n_hyps, (b + 1) * n_hyps)
            T = self.logp[b].shape[0]
            meta = torch.tensor([out_len] * n_hyps + [last[h] for h in hs], dtype=torch.int32)
            meta = torch.cat([meta, cand[b * n_hyps:(b + 1) * n_hyps].reshape(-1).to(torch.int32)])
            ptrs = torch.tensor([r_prev[h].data_ptr() for h in hs], dtype=torch.int64)
            meta_d, ptrs_d = meta.to(self.device), ptrs.to(self.device)
            psi = torch.empty(n_hyps * nc, device=self.device)
            rn = torch.empty(n_hyps, nc, T, 2, device=self.device)
            lib.ea_ctc_prefix_score(T, self.odim, self.blank, self.eos, n_hyps, nc, self.logp[b].data_ptr(),
                                    ptrs_d.data_ptr(), meta_d.data_ptr(), psi.data_ptr(), rn.data_ptr(),
                                    ops.stream())
            idx = cand[b * n_hyps:(b + 1) * n_hyps].to(self.device)
            log_psi[b * n_hyps:(b + 1) * n_hyps].scatter_(1, idx, psi.view(n_hyps, nc))
            r_new.append(rn)
        log_psi[:, self.blank] = self.logzero
        return log_psi - s_prev, (r_new, log_psi, 0, 0, cand[:, :nsc])

    def index_select_state(self, state, best_ids):
        """best_ids (B, W) in each utterance's (n_hyps * O) space -> the selected hypotheses'
        forward variables and prefix scores (a label outside the scored set takes candidate 0's
        variables, as the reference's scoring_idmap fallback does, :206-209)."""
        r_new, log_psi, f_min, f_max, cand = state
        n_hyps = int(r_new[0].shape[0])
        best = best_ids.to(torch.int64).cpu()
        W = int(best.shape[1])
        r_sel, s_idx = [], []
        for b in range(self.batch):
            for w in range(W):
                bid = int(best[b, w])
                h, lab = bid // self.odim, bid % self.odim
                gh = b * n_hyps + h
                row = cand[gh].tolist()
                pos = row.index(lab) if lab in row else 0
                r_sel.append(r_new[b][h, pos])
                s_idx.append(gh * self.odim + lab)
        s_new = log_psi.reshape(-1)[torch.tensor(s_idx, device=self.device)]
        s_new = s_new.view(-1, 1).repeat(1, self.odim)
        return r_sel, s_new, f_min, f_max

    def extend_prob(self, x):
        raise NotImplementedError("CTCPrefixScoreTH.extend_prob: streaming decoding is not built")

    def extend_state(self, state):
        raise NotImplementedError("CTCPrefixScoreTH.extend_state: streaming decoding is not built")
