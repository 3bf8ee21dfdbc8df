"""Validation CER/WER (espnet/nets/e2e_asr_common.py:100-256; espnet2/asr/espnet_model.py:
551-557, 571-575). CPU: the edit distance against editdistance's published known answers,
the product's ErrorCalculator against the oracle restatement on seeded random batches and the
reference's edge cases (empty references, -1 padding, blank/space tokens). GPU: an eval-mode
forward of the HIP model reports cer_ctc / cer / wer equal to the oracle's on the oracle's
own argmaxes (fp32 mode), and None in training mode."""
import random

import numpy as np
import pytest
import torch

from oracle.error_rates import levenshtein, oracle_cer_ctc, oracle_cer_wer

CHARS = ["<blank>", "<unk>", "<space>", "a", "b", "c", "de", "f", "<sos/eos>"]


def _calc(report_cer=True, report_wer=True):
    from espnet_amd.asr.error_calculator import ErrorCalculator
    return ErrorCalculator(CHARS, "<space>", "<blank>", report_cer, report_wer)


@pytest.mark.parametrize("a,b,d", [("kitten", "sitting", 3), ("", "", 0), ("abc", "", 3), ("", "ab", 2),
                                   ("flaw", "lawn", 2), ("intention", "execution", 5),
                                   (["the", "cat"], ["a", "cat", "sat"], 2), ("abc", "abc", 0)])
def test_edit_distance_known_answers(a, b, d):
    from espnet_amd.asr.error_calculator import edit_distance
    assert levenshtein(a, b) == d
    assert edit_distance(a, b) == d


def test_edit_distance_random_matches_oracle():
    from espnet_amd.asr.error_calculator import edit_distance
    rng = random.Random(0)
    for _ in range(300):
        a = [rng.randrange(4) for _ in range(rng.randrange(12))]
        b = [rng.randrange(4) for _ in range(rng.randrange(12))]
        assert edit_distance(a, b) == levenshtein(a, b)


def _batch(rng, B, L, T):
    ys_pad = np.full((B, L), -1, dtype=np.int64)
    for b in range(B):
        n = rng.integers(1, L + 1)
        ys_pad[b, :n] = rng.integers(2, 8, size=n)  # space and word tokens
    att_hat = rng.integers(0, 9, size=(B, L + 1))
    ctc_hat = rng.integers(0, 8, size=(B, T))
    return ys_pad, att_hat, ctc_hat


@pytest.mark.parametrize("seed", range(5))
def test_error_calculator_matches_oracle(seed):
    rng = np.random.default_rng(seed)
    ys_pad, att_hat, ctc_hat = _batch(rng, 6, 9, 20)
    ec = _calc()
    cer, wer = ec(torch.from_numpy(att_hat), torch.from_numpy(ys_pad))
    ocer, ower = oracle_cer_wer(att_hat, ys_pad, CHARS)
    assert cer == pytest.approx(ocer, abs=1e-12) and wer == pytest.approx(ower, abs=1e-12)
    got = ec(torch.from_numpy(ctc_hat), torch.from_numpy(ys_pad), is_ctc=True)
    assert got == pytest.approx(oracle_cer_ctc(ctc_hat, ys_pad, CHARS), abs=1e-12)


def test_error_calculator_edge_cases():
    ec = _calc()
    # hand-derived: ref "a b" -> "ab" (2 chars, 2 words); hyp "a c" cut at the first -1
    ys_pad = torch.tensor([[3, 2, 4, -1]])
    hyp = torch.tensor([[3, 2, 5, 6, 6]])  # tokens past the reference length are ignored
    assert ec(hyp, ys_pad) == (0.5, 0.5)
    # the blank token's text is removed from the attention hypothesis: "ab" vs "a b"
    assert ec(torch.tensor([[3, 0, 4]]), torch.tensor([[3, 2, 4]])) == (0.0, 1.0)
    # CTC: repeats collapse before blanks/spaces drop; multi-character tokens count per char
    ys = torch.tensor([[6, 3, -1]])  # "dea"
    assert ec(torch.tensor([[6, 6, 0, 3, 3, 2]]), ys, is_ctc=True) == 0.0
    assert ec(torch.tensor([[6, 0, 6, 3]]), ys, is_ctc=True) == pytest.approx(2 / 3)
    # utterances whose reference is empty after stripping are skipped; all empty -> None
    assert ec(torch.tensor([[3, 3]]), torch.tensor([[2, -1]]), is_ctc=True) is None
    assert ec(torch.tensor([[3], [4]]), torch.tensor([[2], [4]]), is_ctc=True) == 0.0
    # report switches
    assert _calc(True, False)(hyp, ys_pad) == (0.5, None)
    assert _calc(False, True)(hyp, ys_pad) == (None, 0.5)
    assert _calc(False, False)(hyp, ys_pad) == (None, None)


def test_model_builds_error_calculator():
    from goldens import load
    from test_model_build import build
    cfg, _ = load("tiny_hybrid")
    m = build(cfg)
    assert m.error_calculator is not None and m.error_calculator.report_cer and m.error_calculator.report_wer


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["tiny_hybrid", "tiny_ctc"])
def test_eval_forward_reports_error_rates(name):
    from goldens import load, section
    from oracle.asr_oracle import OracleASR
    from test_model_build import build
    cfg, d = load(name)
    torch.manual_seed(0)
    m = build(cfg)
    w = {k: torch.from_numpy(v) for k, v in section(d, "w").items()}
    m.load_state_dict(w)
    m.prepare("cuda", amp=False)
    inp = {k: torch.from_numpy(v) for k, v in section(d, "in").items()}
    m.eval()  # before any training-mode forward: that would move the BatchNorm running stats
    with torch.no_grad():
        _, stats, _ = m(**inp)
    ora = OracleASR(cfg, w)
    ora.training = False
    with torch.no_grad():
        ora(**{k: v.clone() for k, v in inp.items()})
    toks = m.token_list
    text = inp["text"][:, : int(inp["text_lengths"].max())].numpy()
    ctc_hat = ora.ctc_logits.argmax(-1).numpy()
    # the device argmax over the padded frames equals the oracle's (bit-exact alignment)
    assert np.array_equal(m.ctc.argmax(m._last_encoder_out[0]).cpu().numpy(), ctc_hat)
    want = oracle_cer_ctc(ctc_hat, text, toks)
    assert stats["cer_ctc"].item() == pytest.approx(want, abs=1e-6)
    if cfg["model_conf"]["ctc_weight"] < 1.0:
        att_hat = ora.decoder_out.argmax(-1).numpy()
        ocer, ower = oracle_cer_wer(att_hat, text, toks)
        assert stats["cer"].item() == pytest.approx(ocer, abs=1e-6)
        assert stats["wer"].item() == pytest.approx(ower, abs=1e-6)
    else:
        assert stats["cer"] is None and stats["wer"] is None
    m.train()
    _, stats, _ = m(**inp)
    assert stats["cer_ctc"] is None and stats["cer"] is None and stats["wer"] is None


@pytest.mark.gpu
def test_validate_one_epoch_matches_oracle():
    """Trainer.validate_one_epoch over the tiny hybrid batch split in two minibatches equals
    the batch-size-weighted average of the oracle's eval-mode stats (reporter.py aggregate)."""
    from goldens import load, section
    from oracle.asr_oracle import OracleASR
    from test_model_build import build
    from espnet_amd.train.trainer import Trainer
    cfg, d = load("tiny_hybrid")
    torch.manual_seed(0)
    m = build(cfg)
    w = {k: torch.from_numpy(v) for k, v in section(d, "w").items()}
    m.load_state_dict(w)
    m.prepare("cuda", amp=False)
    inp = {k: torch.from_numpy(v) for k, v in section(d, "in").items()}
    B = inp["speech"].shape[0]
    assert B >= 2
    cut = B // 2
    parts = [{k: v[:cut] for k, v in inp.items()}, {k: v[cut:] for k, v in inp.items()}]
    got = Trainer.validate_one_epoch(m, iter(parts))
    assert m.training
    ora = OracleASR(cfg, w)
    ora.training = False
    sums, wsum = {}, 0
    for p in parts:
        with torch.no_grad():
            _, st, _ = ora(**{k: v.clone() for k, v in p.items()})
        text = p["text"][:, : int(p["text_lengths"].max())].numpy()
        st = {k: float(v) for k, v in st.items()}
        st["cer_ctc"] = oracle_cer_ctc(ora.ctc_logits.argmax(-1).numpy(), text, m.token_list)
        st["cer"], st["wer"] = oracle_cer_wer(ora.decoder_out.argmax(-1).numpy(), text, m.token_list)
        n = p["speech"].shape[0]
        for k, v in st.items():
            sums[k] = sums.get(k, 0.0) + v * n
        wsum += n
    assert set(got) == set(sums)
    for k in sums:
        assert got[k] == pytest.approx(sums[k] / wsum, rel=1e-4, abs=1e-4), k
