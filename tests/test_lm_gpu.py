"""TransformerLM (espnet2/lm/transformer_lm.py) on the HIP path against the reference run on the
same weights (tests/golden/lm_tiny.npz, oracle/make_goldens.py capture_lm): forward logits,
batch_score next-token log-probabilities, and BeamSearch with LM shallow fusion (decoder +
CTC prefix + LM + length bonus, asr_inference.py:140-183) reproducing the reference's n-best."""
import numpy as np
import pytest
import torch

from goldens import load, section

pytestmark = pytest.mark.gpu


def _lm(amp=False):
    from espnet_amd.lm import TransformerLM
    cfg, d = load("lm_tiny")
    lm = TransformerLM(**cfg["lm_conf"])
    lm.load_state_dict({k: torch.from_numpy(v) for k, v in section(d, "w").items()})
    lm.prepare("cuda", amp=amp)
    lm.eval()
    return cfg, d, lm


def test_lm_logits_and_batch_score_match_reference():
    cfg, d, lm = _lm()
    logits, hidden = lm(torch.from_numpy(d["in.ids"]))
    assert hidden is None
    np.testing.assert_allclose(logits.cpu().numpy(), d["out.logits"], atol=1e-4, rtol=1e-4)
    logp, states = lm.batch_score(torch.from_numpy(d["in.ys"]).cuda(), [None] * 4, None)
    np.testing.assert_allclose(logp.cpu().numpy(), d["out.bs_logp"], atol=1e-4, rtol=1e-4)
    assert states == [None] * 4
    one, st = lm.score(torch.from_numpy(d["in.ys"][1]).cuda(), None, None)
    np.testing.assert_allclose(one.cpu().numpy(), d["out.bs_logp"][1], atol=1e-4, rtol=1e-4)


def test_lm_bf16_close():
    cfg, d, lm = _lm(amp=True)
    logits, _ = lm(torch.from_numpy(d["in.ids"]))
    ref = torch.from_numpy(d["out.logits"])
    e = float((logits.cpu() - ref).norm() / ref.norm())
    assert e < 3e-2, e


def test_beam_search_with_lm_fusion_matches_reference():
    from espnet_amd.asr.inference import attention_beam_search
    from test_inference_gpu import _setup
    m, _, inp = _setup()
    cfg, d, lm = _lm()
    for ci, (beam, lb, mlr, cw, lw) in enumerate(cfg["cases"]):
        got = attention_beam_search(m, inp["speech"], inp["speech_lengths"], beam, lb, mlr, ctc_weight=cw, lm=lm,
                                    lm_weight=lw)
        for u, nbest in enumerate(got):
            n = [e["n"] for e in cfg["nbest"] if e["case"] == ci and e["utt"] == u][0]
            assert len(nbest) == n, (ci, u)
            for r, h in enumerate(nbest):
                k = f"c{ci}.u{u}.h{r}"
                assert h.yseq.tolist() == d[k + ".yseq"].tolist(), (ci, u, r)
                np.testing.assert_allclose(float(h.score), float(d[k + ".score"]), rtol=1e-4, atol=1e-3)
                np.testing.assert_allclose(float(h.scores["lm"]), float(d[k + ".lm"]), rtol=1e-4, atol=1e-3)
