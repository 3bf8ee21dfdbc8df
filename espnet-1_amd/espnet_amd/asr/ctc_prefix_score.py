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
scoring (margin > 0 with att_w, :143-153) runs the kernel over the window's frames only
(ea_ctc_prefix_score_win); streaming decoding's extend_prob / extend_state (:222-269) append
frames to the posteriors and extend a hypothesis's forward variables with the blank recursion
(ea_ctc_prefix_extend).
"""
from __future__ import annotations

from typing import List

import torch

from .. import hip_ops as ops
from .._lib import lib

LOGZERO = -10000000000.0


class CTCPrefixScoreTH:
    def __init__(self, x: torch.Tensor, xlens, blank: int, eos: int, margin: int = 0):
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
        self._init_r0()
        self.scoring_num = 0
        self.margin = int(margin)
        if self.margin > 0:  # frame positions for the attention-weighted centre (:57-62)
            self.frame_ids = torch.arange(self.input_length, dtype=self.dtype, device=self.device)

    def _init_r0(self):
        self.r0 = []
        for lp in self.logp:  # initial state: (logzero, cumulative blank log-probability)
            r = torch.full((lp.shape[0], 2), self.logzero, dtype=torch.float32, device=self.device)
            r[:, 1] = torch.cumsum(lp[:, self.blank], 0)
            self.r0.append(r)

    def __call__(self, y: List[torch.Tensor], state, scoring_ids=None, att_w=None):
        n_bh = len(y)
        n_hyps = n_bh // self.batch
        out_len = len(y[0]) - 1
        last = [int(yy[-1]) for yy in y]
        if state is None:
            r_prev = [self.r0[i // n_hyps] for i in range(n_bh)]
            s_prev = torch.zeros(n_bh, 1, device=self.device)
            f_min_prev, f_max_prev = 0, 1
        else:
            r_prev, s_prev, f_min_prev, f_max_prev = state[0], state[1], state[2], state[3]
        # the attention window (:143-153): frames [start, end) around the attended frames
        win = None
        if att_w is not None and self.margin > 0:
            f_arg = torch.matmul(att_w, self.frame_ids)
            f_min = max(int(f_arg.min().cpu()), f_min_prev)
            f_max = max(int(f_arg.max().cpu()), f_max_prev)
            win = (min(f_max_prev, max(f_min - self.margin, out_len, 1)), min(f_max + self.margin, self.input_length))
        else:
            f_min = f_max = 0
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
            if win is None:
                lib.ea_ctc_prefix_score(T, self.odim, self.blank, self.eos, n_hyps, nc, self.logp[b].data_ptr(),
                                        ptrs_d.data_ptr(), meta_d.data_ptr(), psi.data_ptr(), rn.data_ptr(),
                                        ops.stream())
            else:  # (an utterance shorter than the window's end: its own frames only)
                lib.ea_ctc_prefix_score_win(T, self.odim, self.blank, self.eos, n_hyps, nc, self.logp[b].data_ptr(),
                                            ptrs_d.data_ptr(), meta_d.data_ptr(), win[0], min(win[1], T),
                                            psi.data_ptr(), rn.data_ptr(), ops.stream())
            idx = cand[b * n_hyps:(b + 1) * n_hyps].to(self.device)
            log_psi[b * n_hyps:(b + 1) * n_hyps].scatter_(1, idx, psi.view(n_hyps, nc))
            r_new.append(rn)
        log_psi[:, self.blank] = self.logzero
        return log_psi - s_prev, (r_new, log_psi, f_min, f_max, cand[:, :nsc])

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
        """Streaming decoding (:222-242): x (1, T', O) log-posteriors of the utterance so far;
        when longer than the frames held, the new frames are appended (the frames already held
        are kept as they are)."""
        if x.shape[1] <= self.input_length:
            return
        if self.batch != 1:
            raise ValueError("CTCPrefixScoreTH.extend_prob: streaming decoding holds one utterance")
        new = x[0, self.input_length:].to(self.device).float()
        self.logp = [torch.cat([self.logp[0][:self.input_length], new]).contiguous()]
        self.input_length = int(x.shape[1])
        self.xlens = [self.input_length]
        self._init_r0()
        if self.margin > 0:
            self.frame_ids = torch.arange(self.input_length, dtype=self.dtype, device=self.device)

    def extend_state(self, state):
        """Streaming decoding (:244-269): one hypothesis's state (r (T_old, 2), prefix scores,
        f_min, f_max) with r extended to the frames extend_prob appended: r^n logzero, r^b the
        blank recursion continued frame by frame."""
        if state is None:
            return state
        r_prev, s_prev, f_min_prev, f_max_prev = state
        T_old, T = int(r_prev.shape[0]), self.input_length
        if T_old >= T:
            return state
        r = torch.empty(T, 2, dtype=torch.float32, device=self.device)
        lib.ea_ctc_prefix_extend(T_old, T, self.odim, self.blank, self.logp[0].data_ptr(),
                                 r_prev.contiguous().data_ptr(), r.data_ptr(), ops.stream())
        return (r, s_prev, f_min_prev, f_max_prev)
