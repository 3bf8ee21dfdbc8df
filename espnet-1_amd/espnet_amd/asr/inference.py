"""Inference consumers of the trained model, on the same HIP kernels:

* ``ctc_greedy`` — espnet2/asr/ctc.py:119-127 argmax + the greedy CTC collapse (repeats
  merged, blanks dropped) over each utterance's encoder frames.
* ``attention_greedy`` — espnet/nets/beam_search.py:346-432 with beam_size 1, the decoder as
  the only scorer (ctc_weight 0, no LM, no length bonus): a hypothesis grows by the best
  next token (decoder.batch_score, transformer_decoder.py:194-229) until <eos>, with <eos>
  forced at maxlen (post_process, :462-467); maxlen = encoder frames for maxlenratio 0.
  Each utterance is encoded alone, as Speech2Text does (a padded batch would let the
  conformer's depthwise convolution see padding frames).

Both run the model in eval mode (dropout off, BatchNorm running statistics).
"""
from __future__ import annotations

from typing import List, Tuple

import torch


def _collapse(ids, blank=0):
    out, prev = [], None
    for t in ids:
        if t != prev and t != blank:
            out.append(int(t))
        prev = t
    return out


@torch.no_grad()
def ctc_greedy(model, speech: torch.Tensor, speech_lengths: torch.Tensor) -> List[List[int]]:
    was = model.training
    model.eval()
    try:
        res = []
        for b in range(speech.shape[0]):
            le = int(speech_lengths[b])
            enc, olens = model.encode(speech[b:b + 1, :le], speech_lengths[b:b + 1])
            ids = model.ctc.argmax(enc)[0, :int(olens[0])].tolist()
            res.append(_collapse(ids, model.blank_id))
        return res
    finally:
        model.train(was)


@torch.no_grad()
def attention_greedy(model, speech: torch.Tensor, speech_lengths: torch.Tensor, maxlenratio: float = 0.0,
                     minlenratio: float = 0.0) -> List[Tuple[List[int], float]]:
    if minlenratio != 0.0:
        raise NotImplementedError("minlenratio > 0 (beam_search.py retry loop) is not implemented")
    was = model.training
    model.eval()
    try:
        res = []
        sos, eos = model.sos, model.eos
        for b in range(speech.shape[0]):
            le = int(speech_lengths[b])
            enc, olens = model.encode(speech[b:b + 1, :le], speech_lengths[b:b + 1])
            T = enc.shape[1]
            if maxlenratio == 0:
                maxlen = T
            elif maxlenratio < 0:
                maxlen = -1 * int(maxlenratio)
            else:
                maxlen = max(1, int(maxlenratio * T))
            yseq = [sos]
            score = 0.0
            st = [None]  # the decoder's key/value cache row, carried from step to step
            for i in range(maxlen):
                ys = torch.tensor([yseq], dtype=torch.long, device=enc.device)
                logp, st = model.decoder.batch_score(ys, st, enc)
                tok = int(torch.argmax(logp[0]))
                score += float(logp[0, tok])
                yseq.append(tok)
                if i == maxlen - 1 and tok != eos:
                    yseq.append(eos)
                if yseq[-1] == eos:
                    break
            res.append((yseq[1:-1], score))
        return res
    finally:
        model.train(was)


@torch.no_grad()
def attention_beam_search(model, speech: torch.Tensor, speech_lengths: torch.Tensor, beam_size: int,
                          length_bonus: float = 0.0, maxlenratio: float = 0.0, minlenratio: float = 0.0,
                          ctc_weight: float = 0.0, batch: bool = False, lm=None, lm_weight: float = 1.0):
    """Speech2Text-style decoding (espnet2/bin/asr_inference.py:140-175) with BeamSearch
    (espnet/nets/beam_search.py) over the decoder (weight 1 - ctc_weight), the CTC prefix
    scorer (ctc_weight, pre-beam "full") and LengthBonus (length_bonus): per utterance the
    n-best list of Hypothesis records (yseq with <sos>/<eos>, score, per-scorer scores)."""
    from .beam_search import BatchBeamSearch, BeamSearch, CTCPrefixScorer, LengthBonus
    if batch:  # espnet/nets/batch_beam_search.py under its own name (the same batched search)
        BeamSearch = BatchBeamSearch  # noqa: N806
    was = model.training
    model.eval()
    try:
        V = model.vocab_size
        scorers = {"decoder": model.decoder, "ctc": CTCPrefixScorer(model.ctc, model.eos),
                   "length_bonus": LengthBonus(V)}
        weights = {"decoder": 1.0 - ctc_weight, "ctc": ctc_weight, "length_bonus": length_bonus}
        if lm is not None:  # shallow fusion (asr_inference.py:149-183: scorers["lm"], lm_weight)
            scorers["lm"], weights["lm"] = lm, lm_weight
        bs = BeamSearch(scorers=scorers, weights=weights,
                        beam_size=beam_size, vocab_size=V, sos=model.sos, eos=model.eos, pre_beam_score_key="full")
        res = []
        for b in range(speech.shape[0]):
            le = int(speech_lengths[b])
            enc, _ = model.encode(speech[b:b + 1, :le], speech_lengths[b:b + 1])
            res.append(bs(enc[0], maxlenratio=maxlenratio, minlenratio=minlenratio))
        return res
    finally:
        model.train(was)
