"""Beam search over full scorers — drop-in for espnet/nets/beam_search.py:17-483 (BeamSearch,
Hypothesis) with espnet/nets/scorers/length_bonus.py (LengthBonus) and
espnet/nets/e2e_asr_common.py:18-48 (end_detect).

Same constructor arguments, scorer/weight dictionaries, hypothesis record, search order
(per running hypothesis: weighted full scores + previous score, top-k, merge into the
sorted, beam-pruned pool) and end conditions (<eos> forced at maxlen, end detection for
maxlenratio 0, retry with a smaller minlenratio when nothing ended).  MI355X layout: at every
step ALL running hypotheses (they share a length) are scored in ONE batched call per scorer
(the decoder's `batch_score`, HIP kernels over an (n_hyps, T, d) memory); only the
(n_hyps, vocab) score matrix comes back to the host for the selection, which is done in f32
exactly as the reference does it.

Partial scorers (CTCPrefixScorer, pre-beam) are not built yet: passing one raises.
"""
from __future__ import annotations

import math
from typing import Any, Dict, List, NamedTuple, Optional, Union

import torch


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


class BeamSearch(torch.nn.Module):
    """beam_search.py:30-483 for full scorers (decoder, length bonus, LMs with batch_score)."""

    def __init__(self, scorers: Dict[str, Any], weights: Dict[str, float], beam_size: int, vocab_size: int,
                 sos: int, eos: int, token_list: Optional[List[str]] = None, pre_beam_ratio: float = 1.5,
                 pre_beam_score_key: Optional[str] = None, hyp_primer: Optional[List[int]] = None):
        super().__init__()
        self.weights = weights
        self.scorers = {}
        self.full_scorers = {}
        for k, v in scorers.items():
            w = weights.get(k, 0)
            if w == 0 or v is None:
                continue
            if hasattr(v, "score_partial"):
                raise NotImplementedError(f"partial scorer {k!r} (CTC prefix scoring) is not built yet")
            if not hasattr(v, "batch_score"):
                raise TypeError(f"{k} ({type(v)}) has no batch_score")
            self.scorers[k] = v
            self.full_scorers[k] = v
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

    def init_hyp(self, x: torch.Tensor) -> List[Hypothesis]:
        states = {k: (d.init_state(x) if hasattr(d, "init_state") else None) for k, d in self.scorers.items()}
        primer = [self.sos] if self.hyp_primer is None else self.hyp_primer
        return [Hypothesis(score=0.0, scores={k: 0.0 for k in self.scorers}, states=states,
                           yseq=torch.tensor(primer))]

    @staticmethod
    def append_token(xs: torch.Tensor, x: int) -> torch.Tensor:
        return torch.cat((xs, torch.tensor([x], dtype=xs.dtype, device=xs.device)))

    def _score_all(self, running: List[Hypothesis], x: torch.Tensor) -> Dict[str, torch.Tensor]:
        """Every full scorer on every running hypothesis in one batched call:
        {name: (n_hyps, n_vocab) f32 on the host}."""
        n = len(running)
        ys = torch.stack([h.yseq for h in running]).to(x.device)
        xs = x.unsqueeze(0).expand(n, *x.shape)
        out = {}
        for k, d in self.full_scorers.items():
            sc, _ = d.batch_score(ys, [h.states[k] for h in running], xs)
            out[k] = sc.float().cpu()
        return out

    def search(self, running_hyps: List[Hypothesis], x: torch.Tensor) -> List[Hypothesis]:
        """beam_search.py:291-344."""
        best_hyps = []
        allsc = self._score_all(running_hyps, x)
        for hi, hyp in enumerate(running_hyps):
            weighted = torch.zeros(self.n_vocab, dtype=torch.float32)
            scores = {k: allsc[k][hi] for k in self.full_scorers}
            for k in self.full_scorers:
                weighted += self.weights[k] * scores[k]
            weighted += hyp.score
            for j in weighted.topk(self.beam_size)[1].tolist():
                best_hyps.append(Hypothesis(
                    score=weighted[j], yseq=self.append_token(hyp.yseq, j),
                    scores={k: hyp.scores[k] + v[j] for k, v in scores.items()},
                    states=dict(hyp.states)))
            best_hyps = sorted(best_hyps, key=lambda h: h.score, reverse=True)[: min(len(best_hyps), self.beam_size)]
        return best_hyps

    def post_process(self, i: int, maxlen: int, maxlenratio: float, running_hyps: List[Hypothesis],
                     ended_hyps: List[Hypothesis]) -> List[Hypothesis]:
        """beam_search.py:434-482."""
        if i == maxlen - 1:
            running_hyps = [h._replace(yseq=self.append_token(h.yseq, self.eos)) for h in running_hyps]
        remained = []
        for hyp in running_hyps:
            if int(hyp.yseq[-1]) == self.eos:
                for k, d in self.full_scorers.items():
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
