"""Inference consumers: CTC greedy decoding and beam-1 attention
decoding (espnet/nets/beam_search.py with the decoder as the only scorer) through the HIP
model in eval mode, against the oracle (CPU restatement, same weights) — token sequences
bit-exact, hypothesis scores within 1e-3 (fp32 mode)."""
import numpy as np
import pytest
import torch

from goldens import load, section

pytestmark = pytest.mark.gpu


def _setup():
    from oracle.asr_oracle import OracleASR
    from test_model_build import build
    cfg, d = load("tiny_hybrid")
    torch.manual_seed(0)
    m = build(cfg)
    w = {k: torch.from_numpy(v) for k, v in section(d, "w").items()}
    m.load_state_dict(w)
    m.prepare("cuda", amp=False)
    inp = {k: torch.from_numpy(v) for k, v in section(d, "in").items()}
    return m, OracleASR(cfg, w), inp


def test_ctc_greedy_matches_oracle():
    from oracle.asr_oracle import oracle_ctc_greedy
    from espnet_amd.asr.inference import ctc_greedy
    m, ora, inp = _setup()
    got = ctc_greedy(m, inp["speech"], inp["speech_lengths"])
    ref = oracle_ctc_greedy(ora, inp["speech"], inp["speech_lengths"])
    assert got == ref
    assert m.training  # mode restored


def test_attention_greedy_matches_oracle():
    from oracle.asr_oracle import oracle_attention_greedy
    from espnet_amd.asr.inference import attention_greedy
    m, ora, inp = _setup()
    got = attention_greedy(m, inp["speech"], inp["speech_lengths"])
    ref = oracle_attention_greedy(ora, inp["speech"], inp["speech_lengths"])
    for (gs, gsc), (rs, rsc) in zip(got, ref):
        assert gs == rs
        np.testing.assert_allclose(gsc, rsc, rtol=1e-4, atol=1e-3)


def test_decoder_batch_score_matches_full_forward():
    """batch_score over a batch of prefixes == the log-softmax of the last position of the
    training-path decoder (eval mode) on the same prefixes."""
    m, ora, inp = _setup()
    m.eval()
    with torch.no_grad():
        enc, olens = m.encode(inp["speech"][:1, :int(inp["speech_lengths"][0])], inp["speech_lengths"][:1])
        V = m.vocab_size
        ys = torch.randint(1, V - 1, (3, 5))
        ys[:, 0] = m.sos
        xs = enc.expand(3, -1, -1).contiguous()
        logp, states = m.decoder.batch_score(ys.cuda(), [None] * 3, xs)
        full, _ = m.decoder(xs, torch.full((3,), xs.shape[1], dtype=torch.long, device=xs.device), ys.cuda(),
                            torch.full((3,), 5, dtype=torch.long, device=xs.device))
        torch.testing.assert_close(logp, torch.log_softmax(full[:, -1], -1), atol=1e-5, rtol=1e-5)
    assert len(states) == 3 and [s[1] for s in states] == [0, 1, 2]
    cache = states[0][0]
    assert cache.L == 5 and tuple(cache.kv.shape) == (len(m.decoder.decoders), 3, 5, 2 * xs.shape[2])


@pytest.mark.parametrize("graph", [False, True])
@pytest.mark.parametrize("amp", [False, True])
def test_decoder_kv_cache_steps_match_full_forward(amp, graph, monkeypatch):
    """Incremental decoding (transformer_decoder.py:146-229 with its cache): every step's
    batch_score over the previous step's cache rows — gathered in a shuffled order, as a beam
    reorders its hypotheses — equals the full decoder forward of the same prefixes at their
    last position (fp32: 2e-5; bf16: the step and the full pass round the same bf16 operands in
    different GEMM shapes, 2e-2 on the log-probabilities).  graph=True: the captured steps
    (DecodeGraphs: static key/value buffers, position and tokens in device memory)."""
    from test_model_build import build
    from espnet_amd.asr.decoder.transformer_decoder import TransformerDecoder
    monkeypatch.setattr(TransformerDecoder, "decode_graph", graph)
    cfg, d = load("tiny_hybrid")
    torch.manual_seed(0)
    m = build(cfg)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in section(d, "w").items()})
    m.prepare("cuda", amp=amp)
    inp = {k: torch.from_numpy(v) for k, v in section(d, "in").items()}
    m.eval()
    g = torch.Generator().manual_seed(3)
    with torch.no_grad():
        enc, _ = m.encode(inp["speech"][:1, :int(inp["speech_lengths"][0])], inp["speech_lengths"][:1])
        n, V, T = 4, m.vocab_size, enc.shape[1]
        xs = enc.expand(n, -1, -1)
        ys = torch.full((n, 1), m.sos, dtype=torch.long)
        states = [None] * n
        for step in range(7):
            logp, st = m.decoder.batch_score(ys.cuda(), states, xs)
            full, _ = m.decoder(xs.contiguous(), torch.full((n,), T, dtype=torch.long, device="cuda"), ys.cuda(),
                                torch.full((n,), ys.shape[1], dtype=torch.long, device="cuda"))
            ref = torch.log_softmax(full[:, -1].float(), -1)
            tol = 2e-5 if not amp else 2e-2
            torch.testing.assert_close(logp, ref, atol=tol, rtol=tol)
            # next step: shuffled parents (a beam's reordering), each extended by a token
            parents = torch.randperm(n, generator=g)
            ys = torch.cat([ys[parents], torch.randint(2, V - 1, (n, 1), generator=g)], dim=1)
            states = [st[int(p)] for p in parents]
        assert st[0][0].L == 7
        assert (type(st[0][0]).__name__ == "GraphStepKV") == graph
    m.train()


def test_decoder_graph_states_fall_back_past_capacity(monkeypatch):
    """A captured decoding run hands out GraphStepKV states; once a prefix outgrows the run's
    key/value capacity (graph_lcap) batch_score continues on the eager incremental path from
    those states (the run's buffer cropped to the prefix), and a stale state re-builds its
    cache from the prefix.  Every step still equals the full decoder forward (fp32, 2e-5)."""
    from test_model_build import build
    from espnet_amd.asr.decoder.transformer_decoder import DecoderKVCache, GraphStepKV, TransformerDecoder
    monkeypatch.setattr(TransformerDecoder, "decode_graph", True)
    monkeypatch.setattr(TransformerDecoder, "graph_lcap", 4)
    cfg, d = load("tiny_hybrid")
    torch.manual_seed(0)
    m = build(cfg)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in section(d, "w").items()})
    m.prepare("cuda", amp=False)
    inp = {k: torch.from_numpy(v) for k, v in section(d, "in").items()}
    m.eval()
    g = torch.Generator().manual_seed(5)
    kinds = []
    with torch.no_grad():
        enc, _ = m.encode(inp["speech"][:1, :int(inp["speech_lengths"][0])], inp["speech_lengths"][:1])
        n, V, T = 3, m.vocab_size, enc.shape[1]
        xs = enc.expand(n, -1, -1)
        ys = torch.full((n, 1), m.sos, dtype=torch.long)
        states = [None] * n
        for step in range(7):
            logp, st = m.decoder.batch_score(ys.cuda(), states, xs)
            kinds.append(type(st[0][0]).__name__)
            full, _ = m.decoder(xs.contiguous(), torch.full((n,), T, dtype=torch.long, device="cuda"), ys.cuda(),
                                torch.full((n,), ys.shape[1], dtype=torch.long, device="cuda"))
            torch.testing.assert_close(logp, torch.log_softmax(full[:, -1].float(), -1), atol=2e-5, rtol=2e-5)
            parents = torch.randperm(n, generator=g)
            ys = torch.cat([ys[parents], torch.randint(2, V - 1, (n, 1), generator=g)], dim=1)
            states = [st[int(p)] for p in parents]
        assert kinds[:4] == ["GraphStepKV"] * 4 and kinds[4:] == ["DecoderKVCache"] * 3
        # a stale captured state (its run has stepped on since) scores from the prefix
        enc2 = enc.expand(1, -1, -1)
        y1 = torch.full((1, 1), m.sos, dtype=torch.long).cuda()
        _, s1 = m.decoder.batch_score(y1, [None], enc2)
        y2 = torch.cat([y1, torch.full((1, 1), 5, dtype=torch.long, device="cuda")], 1)
        _, s2 = m.decoder.batch_score(y2, s1, enc2)
        assert isinstance(s1[0][0], GraphStepKV) and s1[0][0].step != s1[0][0].run.nstep
        assert TransformerDecoder._as_cache(s1[0][0]) is None
        logp, s3 = m.decoder.score(y2[0], s1[0], enc2[0])
        full, _ = m.decoder(enc2.contiguous(), torch.full((1,), T, dtype=torch.long, device="cuda"), y2,
                            torch.full((1,), 2, dtype=torch.long, device="cuda"))
        torch.testing.assert_close(logp, torch.log_softmax(full[0, -1].float(), -1), atol=2e-5, rtol=2e-5)
        assert isinstance(s3[0], DecoderKVCache)
    m.train()


def test_beam_search_matches_reference_goldens():
    """BeamSearch (decoder + LengthBonus, and joint CTC/attention with the CTC prefix kernel at
    ctc_weight 0.3/0.5; beams 3/4, maxlenratio 0 with end detection and 0.5) on the HIP model: every n-best hypothesis's token sequence equals the reference
    BeamSearch's (tests/golden/beam.npz, oracle/make_goldens.py capture_beam); scores within
    1e-3 (fp32 mode)."""
    from espnet_amd.asr.inference import attention_beam_search
    m, ora, inp = _setup()
    bc, bd = load("beam")
    for ci, case in enumerate(bc["cases"]):
        beam, lb, mlr = case[:3]
        cw = case[3] if len(case) > 3 else 0.0
        got = attention_beam_search(m, inp["speech"], inp["speech_lengths"], beam, lb, mlr, ctc_weight=cw)
        for u, nbest in enumerate(got):
            n = [e["n"] for e in bc["nbest"] if e["case"] == ci and e["utt"] == u][0]
            assert len(nbest) == n
            for r, h in enumerate(nbest):
                k = f"c{ci}.u{u}.h{r}"
                assert h.yseq.tolist() == bd[k + ".yseq"].tolist(), (ci, u, r)
                np.testing.assert_allclose(float(h.score), float(bd[k + ".score"]), rtol=1e-4, atol=1e-3)
                np.testing.assert_allclose(float(h.scores["decoder"]), float(bd[k + ".decoder"]), rtol=1e-4,
                                           atol=1e-3)
                if cw:
                    np.testing.assert_allclose(float(h.scores["ctc"]), float(bd[k + ".ctc"]), rtol=1e-4, atol=1e-3)
    assert m.training


def test_joint_beam_search_runs_in_bf16():
    """The AMP (bf16) model decodes with the joint scorer: n-best lists are sorted, every
    hypothesis is <sos> ... <eos>, and its score equals the weighted sum of its per-scorer
    scores (decoder 0.7, ctc 0.3, length bonus 0.2 per emitted token)."""
    from espnet_amd.asr.inference import attention_beam_search
    from oracle.asr_oracle import OracleASR  # noqa: F401  (same setup as the other tests)
    from test_model_build import build
    cfg, d = load("tiny_hybrid")
    torch.manual_seed(0)
    m = build(cfg)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in section(d, "w").items()})
    m.prepare("cuda", amp=True)
    inp = {k: torch.from_numpy(v) for k, v in section(d, "in").items()}
    res = attention_beam_search(m, inp["speech"], inp["speech_lengths"], 4, length_bonus=0.2, ctc_weight=0.3)
    for nbest in res:
        assert len(nbest) >= 1
        scores = [float(h.score) for h in nbest]
        assert scores == sorted(scores, reverse=True)
        for h in nbest:
            ys = h.yseq.tolist()
            assert ys[0] == m.sos and ys[-1] == m.eos  # (<eos> <eos> when forced at maxlen, as in the reference)
            lb = float(h.scores["length_bonus"])  # emitted tokens (an <eos> forced at maxlen is not scored)
            assert lb in (len(ys) - 1, len(ys) - 2)
            tot = 0.7 * float(h.scores["decoder"]) + 0.3 * float(h.scores["ctc"]) + 0.2 * lb
            np.testing.assert_allclose(float(h.score), tot, rtol=1e-4, atol=1e-3)
            assert np.isfinite(float(h.scores["ctc"]))
