"""Raw-waveform frontend: DefaultFrontend (Stft -> power -> LogMel)
and GlobalMVN against the reference's own modules run under fixed inputs
(tests/golden/frontend.npz, oracle/make_goldens.py).  The mel matrix is librosa's algorithm
restated (librosa is absent here: PARITY UNPINNED against librosa itself; everything
downstream of the mel matrix is pinned to the reference's code path).

Tolerances: the reference's STFT is torch.stft (pocketfft, f32); ours is framing + one exact
f32 DFT-basis GEMM, so spectra agree to f32 rounding of two different summation orders.
Log-mel features are compared with atol 2e-3 (|feat| ~ 5..15), their mean abs error must be
below 1e-4, and every padded frame must be exactly 0."""
import numpy as np
import pytest
import torch

from goldens import load


def _emulated_frontend(x, lens, melmat, n_fft, hop, win_length=None):
    """The HIP algorithm (framing with reflect padding + window, DFT-basis matmul, power,
    mel matmul, log, masks) in f32 torch on the CPU: checks the framing semantics and the
    basis against torch.stft before any GPU is involved."""
    from espnet_amd.asr.frontend.default import Stft
    st = Stft(n_fft=n_fft, win_length=win_length, hop_length=hop)
    win, basis = st._consts(torch.device("cpu"))
    B, Ns = x.shape
    pad = n_fft // 2
    xp = torch.nn.functional.pad(x[:, None], (pad, pad), mode="reflect")[:, 0]
    nF = (Ns + 2 * pad - n_fft) // hop + 1
    frames = xp.unfold(1, n_fft, hop)[:, :nF] * win
    spec = frames.reshape(-1, n_fft) @ basis.t()
    nb = n_fft // 2 + 1
    flens = st.frames_lens(lens)
    pw = (spec[:, :nb] ** 2 + spec[:, nb:] ** 2).view(B, nF, nb)
    pw = pw * (torch.arange(nF)[None, :, None] < flens[:, None, None])
    mel = torch.clamp(pw @ melmat, min=1e-10).log()
    return mel * (torch.arange(nF)[None, :, None] < flens[:, None, None]), flens


def test_mel_filterbank_matches_reference_buffer():
    from espnet_amd.asr.frontend.default import LogMel
    cfg, d = load("frontend")
    for key, conf in cfg["cases"].items():
        lm = LogMel(fs=conf["fs"], n_fft=conf["n_fft"], n_mels=conf["n_mels"], fmin=conf.get("fmin"),
                    fmax=conf.get("fmax"))
        assert np.array_equal(lm.melmat.numpy(), d[f"{key}.melmat"])


@pytest.mark.parametrize("key", ["default", "win400"])
def test_oracle_and_emulation_match_reference(key):
    from oracle.asr_oracle import default_frontend
    cfg, d = load("frontend")
    conf = cfg["cases"][key]
    x, lens = torch.from_numpy(d["x"]), torch.from_numpy(d["lens"])
    melmat = torch.from_numpy(d[f"{key}.melmat"])
    f, fl = default_frontend(x, lens, melmat, n_fft=conf["n_fft"], hop=conf["hop_length"],
                             win_length=conf.get("win_length"))
    assert np.array_equal(fl.numpy(), d[f"{key}.flens"])
    assert np.array_equal(f.numpy(), d[f"{key}.feats"])
    e, el = _emulated_frontend(x, lens, melmat, conf["n_fft"], conf["hop_length"], conf.get("win_length"))
    assert np.array_equal(el.numpy(), d[f"{key}.flens"])
    ref = d[f"{key}.feats"]
    np.testing.assert_allclose(e.numpy(), ref, atol=2e-3)
    assert np.abs(e.numpy() - ref).mean() < 1e-4
    assert (e.numpy()[ref == 0] == 0).all()


def test_oracle_global_mvn_matches_reference():
    from oracle.asr_oracle import global_mvn
    _, d = load("frontend")
    y = global_mvn(torch.from_numpy(d["default.feats"]), torch.from_numpy(d["default.flens"]),
                   torch.from_numpy(d["mvn.mean"]), torch.from_numpy(d["mvn.std"]))
    assert np.array_equal(y.numpy(), d["mvn.y"])


def test_global_mvn_stats_file(tmp_path):
    from espnet_amd.asr.frontend.default import GlobalMVN
    _, d = load("frontend")
    sp = tmp_path / "feats_stats.npz"
    np.savez(sp, count=d["mvn.count"], sum=d["mvn.sum"], sum_square=d["mvn.sum_square"])
    m = GlobalMVN(sp)
    # the reference's forward re-casts its buffers to the input dtype (global_mvn.py:86-87),
    # so the captured ones are f32; ours stay f64 (cast per call)
    assert m.mean.dtype == torch.float64
    assert np.array_equal(m.mean.float().numpy(), d["mvn.mean"]) and np.array_equal(m.std.float().numpy(), d["mvn.std"])
    assert list(dict(m.named_buffers())) == ["mean", "std"]


@pytest.mark.gpu
@pytest.mark.parametrize("key", ["default", "win400"])
def test_frontend_hip_matches_reference(key):
    from espnet_amd.asr.frontend.default import DefaultFrontend
    cfg, d = load("frontend")
    conf = cfg["cases"][key]
    fe = DefaultFrontend(**conf).cuda()
    x, lens = torch.from_numpy(d["x"]).cuda(), torch.from_numpy(d["lens"]).cuda()
    f, fl = fe(x, lens)
    torch.cuda.synchronize()
    ref = d[f"{key}.feats"]
    assert np.array_equal(fl.cpu().numpy(), d[f"{key}.flens"])
    got = f.cpu().numpy()
    np.testing.assert_allclose(got, ref, atol=2e-3)
    assert np.abs(got - ref).mean() < 1e-4
    assert (got[ref == 0] == 0).all()


@pytest.mark.gpu
def test_global_mvn_hip_matches_reference(tmp_path):
    from espnet_amd.asr.frontend.default import GlobalMVN
    _, d = load("frontend")
    sp = tmp_path / "feats_stats.npz"
    np.savez(sp, count=d["mvn.count"], sum=d["mvn.sum"], sum_square=d["mvn.sum_square"])
    m = GlobalMVN(sp)
    y, _ = m(torch.from_numpy(d["default.feats"]).cuda(), torch.from_numpy(d["default.flens"]).cuda())
    torch.cuda.synchronize()
    np.testing.assert_allclose(y.cpu().numpy(), d["mvn.y"], atol=1e-6, rtol=1e-6)


@pytest.mark.gpu
def test_model_with_frontend_matches_feature_model():
    """ESPnetASRModel with frontend=default (raw waveform in) equals the same weights fed the
    oracle's log-mel features of that waveform (input_size set, no frontend): the frontend is
    wired exactly where espnet_model.py:414-431 puts it (before SpecAug / normalisation)."""
    from oracle.asr_oracle import default_frontend
    from espnet_amd.tasks.asr import build_model
    from goldens import section
    cfg, d = load("tiny_hybrid")
    V, F = cfg["vocab_size"], cfg["input_size"]
    tok = ["<blank>", "<unk>"] + [f"t{i}" for i in range(V - 3)] + ["<sos/eos>"]
    fconf = dict(fs=16000, n_fft=512, hop_length=128, n_mels=F)
    base = dict(token_list=tok, encoder="conformer", encoder_conf=cfg["encoder_conf"], decoder="transformer",
                decoder_conf=cfg["decoder_conf"], model_conf=cfg["model_conf"], normalize="utterance_mvn")
    w = {k: torch.from_numpy(v) for k, v in section(d, "w").items()}
    inp = {k: torch.from_numpy(v) for k, v in section(d, "in").items()}
    frames = inp["speech_lengths"]
    slens = (frames - 1) * 128 + 50  # stft frame count (l + 512 - 512) // 128 + 1 == frames
    g = torch.Generator().manual_seed(3)
    wav = torch.randn(len(slens), int(slens.max()), generator=g) * 0.1
    for i, le in enumerate(slens.tolist()):
        wav[i, le:] = 0.0
    losses = []
    for use_fe in (True, False):
        torch.manual_seed(0)
        if use_fe:
            m = build_model(dict(base, frontend="default", frontend_conf=fconf))
            melmat = m.frontend.logmel.melmat.clone()
            m.load_state_dict(dict(w, **{"frontend.logmel.melmat": melmat}))
            batch = dict(speech=wav, speech_lengths=slens, text=inp["text"], text_lengths=inp["text_lengths"])
        else:
            m = build_model(dict(base, input_size=F))
            m.load_state_dict(w)
            feats, fl = default_frontend(wav, slens, melmat, n_fft=512, hop=128)
            assert torch.equal(fl, frames)
            batch = dict(speech=feats, speech_lengths=fl, text=inp["text"], text_lengths=inp["text_lengths"])
        m.prepare("cuda", amp=False)
        m.train()
        loss, stats, _ = m(**batch)
        loss.backward()
        torch.cuda.synchronize()
        losses.append(loss.item())
    np.testing.assert_allclose(losses[0], losses[1], rtol=1e-4)
