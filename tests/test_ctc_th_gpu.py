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


@pytest.mark.parametrize("amp", [False, True])
def test_batch_beam_device_step_matches_host_step(amp, monkeypatch):
    """BatchBeamSearch with the selection on the device (ea_beam_prebeam -> CTC prefix kernel
    -> ea_beam_select, one small record per new hypothesis back to the host) against the same
    search with the reference's host arithmetic (EA_BEAM_DEVICE=0 path): identical n-best
    token sequences, scores within 1e-4 (per-scorer sums are accumulated in float64 on the
    device path, in float32 tensors on the host path)."""
    from espnet_amd.asr.beam_search import BatchBeamSearch, CTCPrefixScorer, LengthBonus
    from test_model_build import build
    from goldens import section
    cfg, d = load("tiny_hybrid")
    torch.manual_seed(0)
    m = build(cfg)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in section(d, "w").items()})
    m.prepare(DEV, amp=amp)
    m.eval()
    inp = {k: torch.from_numpy(v) for k, v in section(d, "in").items()}
    V = m.vocab_size
    # (a fixed output length beyond what an utterance's frames can carry makes every CTC prefix
    # score logzero: the top-k then picks among exact ties at ~-3e9, whose order is the top-k
    # implementation's, on the host as on the device — maxlen stays within the frames here)
    for beam, lb, cw, mlr in ((4, 0.0, 0.3, 0.0), (6, 0.5, 0.5, 0.0), (10, 1.0, 0.3, 0.5)):
        res = {}
        for dev_sel in (False, True):
            monkeypatch.setattr(BatchBeamSearch, "device_select", dev_sel)
            out = []
            for u in range(inp["speech"].shape[0]):
                le = int(inp["speech_lengths"][u])
                enc, _ = m.encode(inp["speech"][u:u + 1, :le], inp["speech_lengths"][u:u + 1])
                bs = BatchBeamSearch(scorers={"decoder": m.decoder, "ctc": CTCPrefixScorer(m.ctc, m.eos),
                                              "length_bonus": LengthBonus(V)},
                                     weights={"decoder": 1.0 - cw, "ctc": cw, "length_bonus": lb}, beam_size=beam,
                                     vocab_size=V, sos=m.sos, eos=m.eos, pre_beam_score_key="full")
                assert (bs._device_plan(enc[0]) is not None) == dev_sel
                out.append(bs(enc[0], maxlenratio=mlr))
            res[dev_sel] = out
        for hu, du in zip(res[False], res[True]):
            assert len(hu) == len(du) and len(du) > 0
            for h, g in zip(hu, du):
                assert h.yseq.tolist() == g.yseq.tolist(), (beam, lb, cw)
                np.testing.assert_allclose(float(g.score), float(h.score), rtol=1e-5, atol=1e-4)
                for k in ("decoder", "ctc"):
                    np.testing.assert_allclose(float(g.scores[k]), float(h.scores[k]), rtol=1e-5, atol=1e-4)
    m.train()


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


def _check(sc, ref, tag):
    mine = sc.cpu().numpy()
    low = ref < -1e9
    assert np.array_equal(mine < -1e9, low), tag
    np.testing.assert_allclose(mine[~low], ref[~low], rtol=1e-5, atol=2e-4, err_msg=tag)


def test_ctc_prefix_score_th_window_matches_reference():
    """margin > 0 with attention weights (ctc_prefix_score.py:57-62, 143-161): the window's
    frame range on the device kernel (ea_ctc_prefix_score_win) vs the reference's scores and
    (f_min, f_max) over three steps (tests/golden/ctc_th_ext.npz)."""
    from espnet_amd.asr.ctc_prefix_score import CTCPrefixScoreTH
    cfg, d = load("ctc_th_ext")
    O, eos, margin = cfg["O"], cfg["eos"], cfg["margin"]
    x = torch.from_numpy(d["w.x"]).to(DEV)
    impl = CTCPrefixScoreTH(x.clone(), torch.from_numpy(d["w.xlens"]), 0, eos, margin=margin)
    state, step = None, 0
    while f"w.s{step}.scores" in d:
        y = [torch.from_numpy(r) for r in d[f"w.s{step}.y"]]
        ids = torch.from_numpy(d[f"w.s{step}.ids"]) if f"w.s{step}.ids" in d else None
        sc, st = impl(y, state, ids, torch.from_numpy(d[f"w.s{step}.att_w"]).to(DEV))
        _check(sc, d[f"w.s{step}.scores"], f"window step {step}")
        assert [st[2], st[3]] == d[f"w.s{step}.fminmax"].tolist()
        if f"w.s{step}.best" not in d:
            break
        state = impl.index_select_state(st, torch.from_numpy(d[f"w.s{step}.best"]))
        step += 1
    assert step == 2


def test_ctc_prefix_score_th_streaming_matches_reference():
    """extend_prob / extend_state (ctc_prefix_score.py:222-269, per hypothesis as
    scorers/ctc.py:128-158 drives them): one utterance revealed 12 -> 20 -> 30 frames, a step
    per chunk, vs the reference's scores; the extended forward variables also equal a scorer
    built on the whole utterance's initial state (a prefix of <sos> only)."""
    from espnet_amd.asr.ctc_prefix_score import CTCPrefixScoreTH
    cfg, d = load("ctc_th_ext")
    O, W, eos, chunks = cfg["O"], cfg["W"], cfg["eos"], cfg["chunks"]
    xs = torch.from_numpy(d["s.x"]).to(DEV)
    impl = CTCPrefixScoreTH(xs[:, :chunks[0]].clone(), torch.tensor([chunks[0]]), 0, eos)
    state, step = None, 0
    for step, tc in enumerate(chunks):
        if step > 0:
            impl.extend_prob(xs[:, :tc].clone())
            per = [impl.extend_state((state[0][i], state[1][i], state[2], state[3])) for i in range(W)]
            assert all(p[0].shape == (tc, 2) for p in per)
            state = ([p[0] for p in per], torch.stack([p[1] for p in per]), per[0][2], per[0][3])
        y = [torch.from_numpy(r) for r in d[f"s.s{step}.y"]]
        sc, st = impl(y, state, None)
        _check(sc, d[f"s.s{step}.scores"], f"streaming step {step}")
        if f"s.s{step}.best" not in d:
            break
        state = impl.index_select_state(st, torch.from_numpy(d[f"s.s{step}.best"]))
    assert step == 2
    # the <sos> state extended from 12 frames equals the 30-frame initial state
    small = CTCPrefixScoreTH(xs[:, :12].clone(), torch.tensor([12]), 0, eos)
    full = CTCPrefixScoreTH(xs.clone(), torch.tensor([30]), 0, eos)
    small.extend_prob(xs.clone())
    r, _, _, _ = small.extend_state((small.r0[0][:12].clone(), None, 0, 1))
    torch.testing.assert_close(r, full.r0[0], rtol=1e-6, atol=1e-5)
