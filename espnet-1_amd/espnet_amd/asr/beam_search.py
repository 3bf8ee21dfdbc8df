"""Beam search over full scorers — drop-in for espnet/nets/beam_search.py:17-483 (BeamSearch,
Hypothesis) with espnet/nets/scorers/length_bonus.py (LengthBonus) and
espnet/nets/e2e_asr_common.py:18-48 (end_detect).

Same constructor arguments, scorer/weight dictionaries, hypothesis record, search order
(per running hypothesis: weighted full scores + previous score, top-k, merge into the
sorted, beam-pruned pool) and end conditions (<eos> forced at maxlen, end detection for
maxlenratio 0, retry with a smaller minlenratio when nothing ended).  MI355X layout: at every
step ALL running hypotheses (they share a length) are scored in ONE batched call per scorer
(the decoder's `batch_score`: one incremental step over a device key/value cache, the
surviving hypotheses' cache rows gathered once per step); only the (n_hyps, vocab) score
matrix comes back to the host for the selection, which is done in f32 exactly as the
reference does it.

Partial scorers (CTCPrefixScorer, scorers/ctc.py) score only the pre-beam candidates of
each hypothesis; every (hypothesis, candidate) pair of a step is scored by ONE launch of the
CTC prefix kernel (csrc/ctc_prefix.hip) on posteriors that stay in HBM.
"""
from __future__ import annotations

import math
import os
from typing import Any, Dict, List, NamedTuple, Optional, Union

import torch

from .. import hip_ops as ops
from .._lib import lib


LOGZERO = -10000000000.0  # ctc_prefix_score.py:33


class Hypothesis(NamedTuple):
    """beam_search.py:17-29."""

    yseq: torch.Tensor
    score: Union[float, torch.Tensor] = 0
    scores: Dict[str, Union[float, torch.Tensor]] = dict()
    states: Dict[str, Any] = dict()

    def asdict(self) -> dict:
        return self._replace(yseq=self.yseq.tolist(), score=float(self.score),
                             scores={k: float(v) for k, v in self.scores.items()})._asdict()


class LengthBonus:
    """scorers/length_bonus.py: +1 per emitted token (weighted by the caller)."""

    def __init__(self, n_vocab: int):
        self.n = n_vocab

    def init_state(self, x):
        return None

    def final_score(self, state):
        return 0.0

    def score(self, y, state, x):
        return torch.tensor([1.0], device=x.device, dtype=x.dtype).expand(self.n), None

    def batch_score(self, ys, states, xs):
        return torch.tensor([1.0], device=xs.device, dtype=xs.dtype).expand(ys.shape[0], self.n), None


def end_detect(ended_hyps, i, M=3, D_end=math.log(1 * math.exp(-10))):
    """e2e_asr_common.py:18-48: stop when, for the last M lengths, the best ended hypothesis
    of that length is far (D_end) below the best overall."""
    if len(ended_hyps) == 0:
        return False
    count = 0
    best_hyp = sorted(ended_hyps, key=lambda x: x["score"], reverse=True)[0]
    for m in range(M):
        same = [x for x in ended_hyps if len(x["yseq"]) == i - m]
        if len(same) > 0:
            best_same = sorted(same, key=lambda x: x["score"], reverse=True)[0]
            if best_same["score"] - best_hyp["score"] < D_end:
                count += 1
    return count == M


class CTCPrefixScorer:
    """scorers/ctc.py:10-97 (CTCPrefixScorer over ctc_prefix_score.py CTCPrefixScore) on the
    device: state of a hypothesis = (prefix score, its (T, 2) forward variables in HBM)."""

    def __init__(self, ctc, eos: int, blank: int = 0):
        self.ctc, self.eos, self.blank = ctc, eos, blank
        self.logp = None

    def init_state(self, x: torch.Tensor):
        """ctc.py:25-37: x (T, d) encoder output of one utterance."""
        lg = self.ctc.logits(x.unsqueeze(0))[0].float().contiguous()
        T, V = lg.shape
        self.logp = torch.empty(T, V, device=x.device)
        r0 = torch.empty(T, 2, device=x.device)
        lib.ea_ctc_prefix_init(T, V, lg.data_ptr(), V, self.blank, self.logp.data_ptr(), r0.data_ptr(), ops.stream())
        return torch.tensor(0.0), r0

    @staticmethod
    def select_state(state, i, new_id=None):
        if len(state) == 5:  # a CTCPrefixScoreTH state (batch_score_partial), ctc.py:40-63
            r_new, log_psi, f_min, f_max, cand = state
            row = cand[i].tolist()
            # an id outside the scored set: scoring_idmap holds -1 there, so the reference
            # indexes the LAST scored column, r[:, :, i, -1] over the snum scored columns
            # (scorers/ctc.py:59-60) — column len(row) - 1, not the appended <eos> column that
            # r_new carries beyond them (ctc_prefix_score.py:92-93)
            pos = row.index(int(new_id)) if int(new_id) in row else len(row) - 1
            return r_new[0][i, pos], log_psi[i, int(new_id)].expand(log_psi.size(1)), f_min, f_max
        sc, st = state
        return sc[i], st[i]

    def batch_init_state(self, x: torch.Tensor):
        """ctc.py:87-99: the vectorised scorer over this utterance's log-posteriors."""
        from .ctc_prefix_score import CTCPrefixScoreTH
        logp = self.ctc.log_softmax(x.unsqueeze(0)).float()
        self.impl = CTCPrefixScoreTH(logp, torch.tensor([logp.size(1)]), 0, self.eos)
        return None

    def batch_score_partial(self, y, ids, state, x):
        """ctc.py:101-126: score the pre-beam ids of every hypothesis in one call."""
        batch_state = (([s[0] for s in state], torch.stack([s[1] for s in state]), state[0][2], state[0][3])
                       if state[0] is not None else None)
        return self.impl(y, batch_state, ids)

    def extend_prob(self, x: torch.Tensor):
        """ctc.py:128-139 (streaming decoding): the encoder output so far -> the vectorised
        scorer's posteriors extended to its frames."""
        logp = self.ctc.log_softmax(x.unsqueeze(0)).float()
        self.impl.extend_prob(logp)

    def extend_state(self, state):
        """ctc.py:141-158: every hypothesis's state extended to the new frames."""
        return [self.impl.extend_state(s) for s in state]

    def final_score(self, state):
        return 0.0

    def score_partial(self, y, ids, state, x):
        """ctc.py:63-80 for one hypothesis."""
        (sc,), (st,) = self.score_partial_multi([y], [ids], [state])
        return sc, st

    def score_partial_multi(self, ys, ids_list, states):
        """score_partial for several hypotheses (same candidate count) in one launch:
        -> ([scores (n_cand,) f32 host], [(prefix scores (n_cand,), r (n_cand, T, 2))])."""
        n, P = len(ys), int(ids_list[0].numel())
        T, V = self.logp.shape
        dev = self.logp.device
        # one small host->device copy: [output lengths | last labels | candidates | r_prev pointers]
        head = [len(y) - 1 for y in ys] + [int(y[-1]) for y in ys]
        cand = torch.cat([i.reshape(-1) for i in ids_list]).to(torch.int32)
        ptrs = torch.tensor([st.data_ptr() for _, st in states], dtype=torch.int64).view(torch.int32)
        nmeta = 2 * n + n * P + (n * P) % 2  # keep the pointer block 8-B aligned
        host = torch.zeros(nmeta + ptrs.numel(), dtype=torch.int32)
        host[:2 * n] = torch.tensor(head, dtype=torch.int32)
        host[2 * n:2 * n + n * P] = cand
        host[nmeta:] = ptrs
        dev_buf = host.to(dev)
        meta_d = dev_buf[:nmeta]
        ptrs_d = dev_buf[nmeta:]
        log_psi = torch.empty(n * P, device=dev)
        r_new = torch.empty(n * P, T, 2, device=dev)
        lib.ea_ctc_prefix_score(T, V, self.blank, self.eos, n, P, self.logp.data_ptr(), ptrs_d.data_ptr(),
                                meta_d.data_ptr(), log_psi.data_ptr(), r_new.data_ptr(), ops.stream())
        psi = log_psi.cpu()
        scores, new_states = [], []
        for h in range(n):
            presub = psi[h * P:(h + 1) * P]
            scores.append(presub - states[h][0])  # ctc.py:76-79: prefix score increment (f32)
            new_states.append((presub, r_new[h * P:(h + 1) * P]))
        return scores, new_states


class BeamSearch(torch.nn.Module):
    """beam_search.py:30-483: full scorers (decoder, length bonus) and partial scorers (CTC prefix)."""

    def __init__(self, scorers: Dict[str, Any], weights: Dict[str, float], beam_size: int, vocab_size: int,
                 sos: int, eos: int, token_list: Optional[List[str]] = None, pre_beam_ratio: float = 1.5,
                 pre_beam_score_key: Optional[str] = None, hyp_primer: Optional[List[int]] = None):
        super().__init__()
        self.weights = weights
        self.scorers = {}
        self.full_scorers = {}
        self.part_scorers = {}
        for k, v in scorers.items():
            w = weights.get(k, 0)
            if w == 0 or v is None:
                continue
            self.scorers[k] = v
            if hasattr(v, "score_partial"):
                if not hasattr(v, "score_partial_multi"):
                    raise TypeError(f"{k} ({type(v)}) has no score_partial_multi")
                self.part_scorers[k] = v
            elif hasattr(v, "batch_score"):
                self.full_scorers[k] = v
            else:
                raise TypeError(f"{k} ({type(v)}) has no batch_score")
        self.sos, self.eos = sos, eos
        self.hyp_primer = hyp_primer
        self.token_list = token_list
        self.pre_beam_size = int(pre_beam_ratio * beam_size)
        self.beam_size = beam_size
        self.n_vocab = vocab_size
        if pre_beam_score_key is not None and pre_beam_score_key != "full" \
                and pre_beam_score_key not in self.full_scorers:
            raise KeyError(f"{pre_beam_score_key} is not found in {self.full_scorers}")
        self.pre_beam_score_key = pre_beam_score_key
        self.do_pre_beam = (pre_beam_score_key is not None and self.pre_beam_size < self.n_vocab
                            and len(self.part_scorers) > 0)

    def init_hyp(self, x: torch.Tensor) -> List[Hypothesis]:
        states = {k: (d.init_state(x) if hasattr(d, "init_state") else None) for k, d in self.scorers.items()}
        primer = [self.sos] if self.hyp_primer is None else self.hyp_primer
        return [Hypothesis(score=0.0, scores={k: 0.0 for k in self.scorers}, states=states,
                           yseq=torch.tensor(primer))]

    @staticmethod
    def append_token(xs: torch.Tensor, x: int) -> torch.Tensor:
        return torch.cat((xs, torch.tensor([x], dtype=xs.dtype, device=xs.device)))

    def _score_all(self, running: List[Hypothesis], x: torch.Tensor):
        """Every full scorer on every running hypothesis in one batched call:
        ({name: (n_hyps, n_vocab) f32 on the host}, {name: per-hypothesis states after the
        call, or None}) — the decoder's state is its row of the step's key/value cache."""
        n = len(running)
        ys = torch.stack([h.yseq for h in running]).to(x.device)
        xs = x.unsqueeze(0).expand(n, *x.shape)
        out, states = {}, {}
        for k, d in self.full_scorers.items():
            sc, st = d.batch_score(ys, [h.states[k] for h in running], xs)
            out[k] = sc.float().cpu()
            states[k] = st
        return out, states

    def beam(self, weighted_scores: torch.Tensor, ids: torch.Tensor):
        """beam_search.py:209-237: top-k full ids and the matching pre-beam (local) ids."""
        if weighted_scores.size(0) == ids.size(0):
            top_ids = weighted_scores.topk(self.beam_size)[1]
            return top_ids, top_ids
        tmp = weighted_scores[ids]
        weighted_scores[:] = -float("inf")
        weighted_scores[ids] = tmp
        top_ids = weighted_scores.topk(self.beam_size)[1]
        local_ids = weighted_scores[ids].topk(self.beam_size)[1]
        return top_ids, local_ids

    def search(self, running_hyps: List[Hypothesis], x: torch.Tensor) -> List[Hypothesis]:
        """beam_search.py:291-344 for all running hypotheses at once: the scorers run batched
        (full scorers, then the partial scorers on each hypothesis's pre-beam), the reference's
        per-hypothesis arithmetic runs row-wise on the (n_hyps, vocab) host scores, and its
        incremental sort-and-prune is one stable descending sort of the n_hyps x beam
        candidates in hypothesis order (it keeps the same beam, ties included)."""
        n, V = len(running_hyps), self.n_vocab
        allsc, allst = self._score_all(running_hyps, x)
        W = torch.zeros(n, V, dtype=torch.float32)
        for k in self.full_scorers:
            W += self.weights[k] * allsc[k]
        if self.do_pre_beam:
            pre = W if self.pre_beam_score_key == "full" else allsc[self.pre_beam_score_key]
            ids = torch.topk(pre, self.pre_beam_size, dim=1)[1]
        else:
            ids = torch.arange(V).expand(n, V)
        part = {k: d.score_partial_multi([h.yseq for h in running_hyps], list(ids),
                                         [h.states[k] for h in running_hyps])
                for k, d in self.part_scorers.items()}
        for k in self.part_scorers:
            W.scatter_(1, ids, W.gather(1, ids) + self.weights[k] * torch.stack(part[k][0]))
        W += torch.stack([torch.as_tensor(h.score, dtype=torch.float32) for h in running_hyps]).view(n, 1)
        if ids.shape[1] == V:  # beam(): no pre-beam
            top = W.topk(self.beam_size, dim=1)[1]
            local = top
        else:  # beam(): pruned candidates masked out
            Wm = torch.full_like(W, -float("inf"))
            Wm.scatter_(1, ids, W.gather(1, ids))
            W = Wm
            top = W.topk(self.beam_size, dim=1)[1]
            local = W.gather(1, ids).topk(self.beam_size, dim=1)[1]
        cand = W.gather(1, top).reshape(-1)
        order = torch.sort(cand, descending=True, stable=True)[1][: self.beam_size].tolist()
        best_hyps = []
        for o in order:
            hi, r = divmod(o, self.beam_size)
            hyp = running_hyps[hi]
            j, pj = int(top[hi, r]), int(local[hi, r])
            new_scores = {k: hyp.scores[k] + allsc[k][hi, j] for k in self.full_scorers}
            new_scores.update({k: hyp.scores[k] + part[k][0][hi][pj] for k in self.part_scorers})
            # beam_search.py:330 merge_states: a full scorer's state after scoring hyp
            new_states = {k: (hyp.states[k] if allst[k] is None else allst[k][hi]) for k in self.full_scorers}
            new_states.update({k: d.select_state(part[k][1][hi], pj) for k, d in self.part_scorers.items()})
            best_hyps.append(Hypothesis(score=W[hi, j], yseq=self.append_token(hyp.yseq, j), scores=new_scores,
                                        states=new_states))
        return best_hyps

    def post_process(self, i: int, maxlen: int, maxlenratio: float, running_hyps: List[Hypothesis],
                     ended_hyps: List[Hypothesis]) -> List[Hypothesis]:
        """beam_search.py:434-482."""
        if i == maxlen - 1:
            running_hyps = [h._replace(yseq=self.append_token(h.yseq, self.eos)) for h in running_hyps]
        remained = []
        for hyp in running_hyps:
            if int(hyp.yseq[-1]) == self.eos:
                for k, d in list(self.full_scorers.items()) + list(self.part_scorers.items()):
                    s = d.final_score(hyp.states[k]) if hasattr(d, "final_score") else 0.0
                    hyp.scores[k] += s
                    hyp = hyp._replace(score=hyp.score + self.weights[k] * s)
                ended_hyps.append(hyp)
            else:
                remained.append(hyp)
        return remained

    @torch.no_grad()
    def forward(self, x: torch.Tensor, maxlenratio: float = 0.0, minlenratio: float = 0.0) -> List[Hypothesis]:
        """beam_search.py:346-432: x (T, d) encoder output of one utterance."""
        if maxlenratio == 0:
            maxlen = x.shape[0]
        elif maxlenratio < 0:
            maxlen = -1 * int(maxlenratio)
        else:
            maxlen = max(1, int(maxlenratio * x.size(0)))
        running = self.init_hyp(x)
        ended: List[Hypothesis] = []
        for i in range(maxlen):
            best = self.search(running, x)
            running = self.post_process(i, maxlen, maxlenratio, best, ended)
            if maxlenratio == 0.0 and end_detect([h.asdict() for h in ended], i):
                break
            if len(running) == 0:
                break
        nbest = sorted(ended, key=lambda h: h.score, reverse=True)
        if len(nbest) == 0:
            return [] if minlenratio < 0.1 else self.forward(x, maxlenratio, max(0.0, minlenratio - 0.1))
        return nbest


class BatchBeamSearch(BeamSearch):
    """espnet/nets/batch_beam_search.py:26-348 (BatchBeamSearch).  The scoring is batched as in
    BeamSearch above (decoder over its key/value cache, one CTC prefix launch per step); what
    differs is the reference's selection rule, reproduced here:
      * partial scores are full-vocabulary rows as CTCPrefixScoreTH returns them: the pre-beam
        ids scored, <eos> ALWAYS scored with the full-sequence probability (TH sets it for every
        hypothesis, ctc_prefix_score.py:178-179), blank and everything else logzero - prefix;
      * the new beam is the global top-k over the flattened (n_hyps x vocab) weighted scores
        (batch_beam, :81-101), in topk order, with no final-score step in post_process."""

    def search(self, running_hyps: List[Hypothesis], x: torch.Tensor) -> List[Hypothesis]:
        n, V = len(running_hyps), self.n_vocab
        allsc, allst = self._score_all(running_hyps, x)
        W = torch.zeros(n, V, dtype=torch.float32)
        for k in self.full_scorers:
            W += self.weights[k] * allsc[k]
        if self.do_pre_beam:
            pre = W if self.pre_beam_score_key == "full" else allsc[self.pre_beam_score_key]
            ids = torch.topk(pre, self.pre_beam_size, dim=1)[1]
        else:
            ids = torch.arange(V).expand(n, V)
        if ids.shape[1] < V:  # <eos> scored for every hypothesis (a duplicate column if pre-beamed)
            ids = torch.cat([ids, torch.full((n, 1), self.eos, dtype=ids.dtype)], dim=1)
        part, pos = {}, {}
        for k, d in self.part_scorers.items():
            sc, st = d.score_partial_multi([h.yseq for h in running_hyps], list(ids),
                                           [h.states[k] for h in running_hyps])
            full = torch.full((n, V), LOGZERO, dtype=torch.float32)
            full -= torch.stack([torch.as_tensor(h.states[k][0], dtype=torch.float32) for h in running_hyps]).view(n, 1)
            full.scatter_(1, ids, torch.stack(sc))
            part[k] = (full, st)
            W += self.weights[k] * full
        W += torch.stack([torch.as_tensor(h.score, dtype=torch.float32) for h in running_hyps]).view(n, 1)
        top = W.view(-1).topk(self.beam_size)[1]
        best_hyps = []
        for t in top.tolist():
            hi, j = divmod(t, V)
            hyp = running_hyps[hi]
            new_scores = {k: hyp.scores[k] + allsc[k][hi, j] for k in self.full_scorers}
            new_scores.update({k: hyp.scores[k] + part[k][0][hi, j] for k in self.part_scorers})
            new_states = {k: (hyp.states[k] if allst[k] is None else allst[k][hi]) for k in self.full_scorers}
            row = ids[hi].tolist()
            pj = row.index(j) if j in row else 0  # TH's scoring_idmap fallback
            new_states.update({k: d.select_state(part[k][1][hi], pj) for k, d in self.part_scorers.items()})
            best_hyps.append(Hypothesis(score=W[hi, j], yseq=self.append_token(hyp.yseq, j), scores=new_scores,
                                        states=new_states))
        return best_hyps

    def post_process(self, i: int, maxlen: int, maxlenratio: float, running_hyps: List[Hypothesis],
                     ended_hyps: List[Hypothesis]) -> List[Hypothesis]:
        """batch_beam_search.py:303-348: <eos> forced at maxlen, ended hypotheses moved out (no
        final-score step)."""
        if i == maxlen - 1:
            running_hyps = [h._replace(yseq=self.append_token(h.yseq, self.eos)) for h in running_hyps]
        remained = []
        for hyp in running_hyps:
            (ended_hyps if int(hyp.yseq[-1]) == self.eos else remained).append(hyp)
        return remained

    # ------------------------------------------------------------------ device-resident steps
    # EA_BEAM_DEVICE=0 keeps the host selection (A/B, and the reference's arithmetic on the host)
    device_select = os.environ.get("EA_BEAM_DEVICE", "1") != "0"

    def _device_plan(self, x):
        """The joint decoding the device step covers: one decoder-like full scorer (batch_score
        -> (n, V) log-probabilities), an optional LengthBonus, one CTCPrefixScorer as the only
        partial scorer, pre-beam on the full weighted scores.  None otherwise."""
        if not (self.device_select and x.is_cuda and self.do_pre_beam and self.pre_beam_score_key == "full"
                and self.hyp_primer is None):
            return None
        if len(self.part_scorers) != 1:
            return None
        (ck, ctc), = self.part_scorers.items()
        if not isinstance(ctc, CTCPrefixScorer):
            return None
        dec = [k for k, d in self.full_scorers.items() if not isinstance(d, LengthBonus)]
        lb = [k for k, d in self.full_scorers.items() if isinstance(d, LengthBonus)]
        if len(dec) != 1 or len(lb) > 1:
            return None
        nc = self.pre_beam_size + 1
        if self.beam_size * nc > 4096 or self.n_vocab > 32768:
            return None
        return dec[0], (lb[0] if lb else None), ck

    @torch.no_grad()
    def forward(self, x: torch.Tensor, maxlenratio: float = 0.0, minlenratio: float = 0.0) -> List[Hypothesis]:
        plan = self._device_plan(x)
        if plan is None:
            return super().forward(x, maxlenratio, minlenratio)
        return self._forward_device(x, maxlenratio, minlenratio, *plan)

    def _forward_device(self, x, maxlenratio, minlenratio, dk, lk, ck):
        """batch_beam_search.py:170-205 + beam_search.py:346-432 with the per-step selection on
        the device: the decoder's (n, V) log-probabilities never leave HBM; per step ONE
        small record per new hypothesis (parent, token, scores) comes back to the host, which
        keeps the reference's hypothesis bookkeeping (yseq, per-scorer scores, <eos> handling,
        end detection)."""
        if maxlenratio == 0:
            maxlen = x.shape[0]
        elif maxlenratio < 0:
            maxlen = -1 * int(maxlenratio)
        else:
            maxlen = max(1, int(maxlenratio * x.size(0)))
        dec, ctc = self.full_scorers[dk], self.part_scorers[ck]
        w_dec, w_ctc = float(self.weights[dk]), float(self.weights[ck])
        w_lb, use_lb = (float(self.weights[lk]), 1) if lk is not None else (0.0, 0)
        K, P, V = self.beam_size, self.pre_beam_size, self.n_vocab
        Pc = P + 1
        dev = x.device
        running = self.init_hyp(x)  # CTC init_state: log-posteriors + r0 on the device
        T = ctc.logp.shape[0]
        i32, f32 = torch.int32, torch.float32
        cand = torch.empty(K * Pc, dtype=i32, device=dev)
        psi = torch.empty(K * Pc, dtype=f32, device=dev)
        r_buf = [torch.empty(K * Pc, T, 2, dtype=f32, device=dev) for _ in range(2)]
        rec = torch.empty(8 * K, dtype=i32, device=dev)  # [rec_i (4K) | rec_f (4K) as f32 bits]
        rec_host = torch.empty(8 * K, dtype=i32).pin_memory()
        cur_st = dict(last=torch.full((K,), self.sos, dtype=i32, device=dev),
                      rptr=torch.zeros(K, dtype=torch.int64, device=dev),
                      prefix=torch.zeros(K, dtype=f32, device=dev), score=torch.zeros(K, dtype=f32, device=dev))
        cur_st["rptr"][0] = running[0].states[ck][1].data_ptr()
        nxt_st = {k: torch.empty_like(v) for k, v in cur_st.items()}
        xs1 = x.unsqueeze(0)
        ended: List[Hypothesis] = []
        buf = 0
        for i in range(maxlen):
            n = len(running)
            ys = torch.stack([h.yseq for h in running])  # host: the decoder reads the last tokens
            logp, dstates = dec.batch_score(ys, [h.states[dk] for h in running], xs1.expand(n, *x.shape))
            logp = logp.float()
            if not logp.is_contiguous():
                logp = logp.contiguous()
            r_new = r_buf[buf]
            lib.ea_beam_prebeam(n, V, logp.data_ptr(), V, w_dec, w_lb, use_lb, P, self.eos, cand.data_ptr(),
                                ops.stream())
            lib.ea_ctc_prefix_score_dev(T, V, ctc.blank, self.eos, n, Pc, ctc.logp.data_ptr(),
                                        cur_st["rptr"].data_ptr(), i, cur_st["last"].data_ptr(), cand.data_ptr(),
                                        psi.data_ptr(), r_new.data_ptr(), ops.stream())
            lib.ea_beam_select(n, V, P, K, T, logp.data_ptr(), V, cand.data_ptr(), psi.data_ptr(),
                               cur_st["prefix"].data_ptr(), cur_st["score"].data_ptr(), w_dec, w_lb, use_lb, w_ctc,
                               r_new.data_ptr(), rec.data_ptr(), rec.data_ptr() + 16 * K, nxt_st["last"].data_ptr(),
                               nxt_st["rptr"].data_ptr(), nxt_st["prefix"].data_ptr(), nxt_st["score"].data_ptr(),
                               ops.stream())
            rec_host.copy_(rec)  # the one device -> host read of the step
            ri = rec_host[:4 * K].view(K, 4).tolist()
            rf = rec_host[4 * K:].view(f32).view(K, 4).tolist()
            best = []
            for b in range(K):
                hi, j, k, empty = ri[b]
                if empty:
                    raise RuntimeError("beam step left fewer candidates than the beam")
                tot, dsc, inc, ps = rf[b]
                hyp = running[hi]
                sc = dict(hyp.scores)
                sc[dk] = hyp.scores[dk] + dsc
                sc[ck] = hyp.scores[ck] + inc
                if lk is not None:
                    sc[lk] = hyp.scores[lk] + 1.0
                st = {dk: dstates[hi], ck: (ps, None)}
                if lk is not None:
                    st[lk] = None
                best.append(Hypothesis(score=tot, yseq=self.append_token(hyp.yseq, j), scores=sc, states=st))
            running = self.post_process(i, maxlen, maxlenratio, best, ended)
            if maxlenratio == 0.0 and end_detect([h.asdict() for h in ended], i):
                break
            if len(running) == 0:
                break
            if len(running) < K:  # ended hypotheses leave the beam: keep the survivors' rows
                alive = [b for b, h in enumerate(best) if int(h.yseq[-1]) != self.eos]
                idx = torch.tensor(alive, dtype=torch.long).to(dev, non_blocking=True)
                for key in cur_st:
                    torch.index_select(nxt_st[key], 0, idx, out=cur_st[key][:len(alive)])
            else:
                cur_st, nxt_st = nxt_st, cur_st
            buf ^= 1
        nbest = sorted(ended, key=lambda h: h.score, reverse=True)
        if len(nbest) == 0:
            return [] if minlenratio < 0.1 else self.forward(x, maxlenratio, max(0.0, minlenratio - 0.1))
        return nbest

