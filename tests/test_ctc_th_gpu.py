"""CTCPrefixScoreTH (espnet/nets/ctc_prefix_score.py:11-270) on the device prefix kernel vs the
reference run on the same log-posteriors (tests/golden/ctc_th.npz, oracle/make_goldens.py
capture_ctc_th): three steps (full vocabulary, pre-beam subset, full) with index_select_state
between them; and the reference BatchBeamSearch's n-best lists (tests/golden/beam_batch.npz)
reproduced by BatchBeamSearch on the HIP model."""
import numpy as np
import pytest
import torch

from goldens import load

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def test_ctc_prefix_score_th_matches_reference():
    from espnet_amd.asr.ctc_prefix_score import CTCPrefixScoreTH
    cfg, d = load("ctc_th")
    B, O, W, eos = cfg["B"], cfg["O"], cfg["W"], cfg["eos"]
    x = torch.from_numpy(d["x"]).to(DEV)
    impl = CTCPrefixScoreTH(x.clone(), torch.from_numpy(d["xlens"]), 0, eos)
    state = None
    step = 0
    while f"s{step}.scores" in d:
        y = [torch.from_numpy(r) for r in d[f"s{step}.y"]]
        ids = torch.from_numpy(d[f"s{step}.ids"]) if f"s{step}.ids" in d else None
        sc, st = impl(y, state, ids)
        ref = d[f"s{step}.scores"]
        mine = sc.cpu().numpy()
        low = ref < -1e9
        assert np.array_equal(mine < -1e9, low), step
        np.testing.assert_allclose(mine[~low], ref[~low], rtol=1e-5, atol=2e-4, err_msg=f"step {step}")
        if f"s{step}.best" not in d:
            break
        state = impl.index_select_state(st, torch.from_numpy(d[f"s{step}.best"]))
        step += 1
    assert step == 2


def test_batch_beam_search_matches_reference_batch_goldens():
    from espnet_amd.asr.inference import attention_beam_search
    from test_inference_gpu import _setup
    m, _, inp = _setup()
    bc, bd = load("beam_batch")
    for ci, case in enumerate(bc["cases"]):
        beam, lb, mlr, cw = case
        got = attention_beam_search(m, inp["speech"], inp["speech_lengths"], beam, lb, mlr, ctc_weight=cw,
                                    batch=True)
        for u, nbest in enumerate(got):
            n = [e["n"] for e in bc["nbest"] if e["case"] == ci and e["utt"] == u][0]
            assert len(nbest) == n, (ci, u)
            for r, h in enumerate(nbest):
                k = f"c{ci}.u{u}.h{r}"
                assert h.yseq.tolist() == bd[k + ".yseq"].tolist(), (ci, u, r)
                np.testing.assert_allclose(float(h.score), float(bd[k + ".score"]), rtol=1e-4, atol=1e-3)


def test_ctc_scorer_batch_api_matches_th():
    """CTCPrefixScorer.batch_init_state / batch_score_partial / select_state (scorers/ctc.py:
    40-126, the interface the reference's BatchBeamSearch drives) agree with CTCPrefixScoreTH
    called directly on the same utterance."""
    from espnet_amd.asr.beam_search import CTCPrefixScorer
    from espnet_amd.asr.ctc_prefix_score import CTCPrefixScoreTH
    from test_inference_gpu import _setup
    m, _, inp = _setup()
    m.eval()
    enc, _ = m.encode(inp["speech"][:1], inp["speech_lengths"][:1])
    x = enc[0]
    sc = CTCPrefixScorer(m.ctc, m.eos)
    assert sc.batch_init_state(x) is None
    y = [torch.tensor([m.sos]), torch.tensor([m.sos])]
    ids = torch.tensor([[3, 4, 5], [5, 6, 7]])
    s1, st1 = sc.batch_score_partial(y, ids, [None, None], x)
    ref = CTCPrefixScoreTH(m.ctc.log_softmax(x.unsqueeze(0)).float(), torch.tensor([x.shape[0]]), 0, m.eos)
    s2, st2 = ref(y, None, ids)
    assert torch.equal(s1, s2)
    # select hypothesis 1's label 6 and continue one step
    hs = [sc.select_state(st1, 1, 6), sc.select_state(st1, 0, 4)]
    y2 = [torch.tensor([m.sos, 6]), torch.tensor([m.sos, 4])]
    s3, _ = sc.batch_score_partial(y2, ids, hs, x)
    O = s2.shape[1]
    r_sel, s_new, _, _ = ref.index_select_state(st2, torch.tensor([[1 * O + 6, 0 * O + 4]]))
    s4, _ = ref(y2, (r_sel, s_new, 0, 0), ids)
    assert torch.equal(s3, s4)
    m.train()
