"""The HIP training step (Trainer.train_one_step: forward, backward, clip_grad_norm_(5),
Adam + WarmupLR on device, zero_grad) against the reference's 2-step trainer golden
(oracle/make_goldens.py capture_train: espnet2/train/trainer.py:567-701), eagerly and as a
captured/replayed hipGraph (espnet_amd/train/graph.py); graph replay vs eager bit-equality
with dropout on; and the non-finite-norm skip (trainer.py:662-697)."""
import numpy as np
import pytest
import torch

from goldens import load, section

pytestmark = pytest.mark.gpu


def _setup(cfg_over=None, dropout=None, amp=False):
    from test_model_build import build
    from espnet_amd.optim.adam import ArenaAdam
    from espnet_amd.schedulers.warmup_lr import WarmupLR
    meta, d = load("train2")
    cfg, _ = load(meta["cfg_name"])
    if dropout is not None:
        cfg = dict(cfg)
        cfg["encoder_conf"] = dict(cfg["encoder_conf"], dropout_rate=dropout, positional_dropout_rate=dropout,
                                   attention_dropout_rate=dropout)
        cfg["decoder_conf"] = dict(cfg["decoder_conf"], dropout_rate=dropout, positional_dropout_rate=dropout,
                                   self_attention_dropout_rate=dropout, src_attention_dropout_rate=dropout)
    torch.manual_seed(0)
    m = build(cfg)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in section(d, "w").items()})
    m.prepare("cuda:0", amp=amp, seed=77)
    m.train()
    opt = ArenaAdam(m, lr=meta["lr"], weight_decay=meta["weight_decay"])
    sched = WarmupLR(opt, warmup_steps=meta["warmup_steps"])
    return meta, d, m, opt, sched


def _check_golden(meta, d, m, outs, opt):
    for s, (loss, gn) in enumerate(outs):
        np.testing.assert_allclose(loss, d[f"out{s}.loss"], rtol=2e-6, atol=1e-4)
        np.testing.assert_allclose(gn, d[f"out{s}.grad_norm"], rtol=1e-4)
    assert opt.step_count == meta["steps"]
    # the last update used the lr the scheduler produced after the previous step
    np.testing.assert_allclose(opt.last_lr(), d[f"out{meta['steps'] - 2}.lr_after"], rtol=1e-6)
    sd = m.state_dict()
    for k, v in section(d, "w_after").items():
        # tolerance as tests/test_oracle_goldens.py::test_oracle_train_two_steps (Adam's
        # sign-like update of near-zero gradient elements; BN-fed depthwise bias)
        tol = 6e-4 if k.endswith("depthwise_conv.bias") else 5e-5
        np.testing.assert_allclose(sd[k].detach().cpu().float().numpy(), v, atol=tol, rtol=1e-5, err_msg=k)


def test_trainer_two_steps_matches_golden_eager():
    from espnet_amd.train.trainer import Trainer
    meta, d, m, opt, sched = _setup()
    outs = []
    for s in range(meta["steps"]):
        batch = {k: torch.from_numpy(v) for k, v in section(d, f"in{s}").items()}
        loss, stats, weight, gn = Trainer.train_one_step(m, batch, opt, sched, grad_clip=meta["grad_clip"])
        outs.append((float(loss), float(gn)))
    _check_golden(meta, d, m, outs, opt)


def test_trainer_two_steps_matches_golden_captured():
    from espnet_amd.train.graph import CapturedTrainStep
    meta, d, m, opt, sched = _setup()
    run = CapturedTrainStep(m, opt, sched, grad_clip=meta["grad_clip"], warmup=1)
    outs = []
    for s in range(meta["steps"]):
        batch = {k: torch.from_numpy(v) for k, v in section(d, f"in{s}").items()}
        loss, stats, weight, gn = run(batch)
        outs.append((float(loss), float(gn)))
    assert len(run.graphs) == 1  # step 0 eager, step 1 captured + replayed
    _check_golden(meta, d, m, outs, opt)


def _batches(d, n):
    base = {k: torch.from_numpy(v) for k, v in section(d, "in0").items()}
    g = torch.Generator().manual_seed(5)
    out = []
    for i in range(n):
        b = dict(base)
        b["speech"] = torch.randn(base["speech"].shape, generator=g)
        b["text"] = torch.where(base["text"] >= 0, torch.randint(2, 48, base["text"].shape, generator=g),
                                base["text"])
        out.append(b)
    return out


@pytest.mark.parametrize("amp", [False, True])
def test_graph_replay_equals_eager_with_dropout(amp):
    """Same init, same batches, dropout 0.1 everywhere: a captured-and-replayed step draws
    the same per-step masks (device salt) and gives bit-identical parameters."""
    from espnet_amd.train.graph import CapturedTrainStep
    from espnet_amd.train.trainer import Trainer
    batches = _batches(load("train2")[1], 4)
    meta, d, m1, o1, s1 = _setup(dropout=0.1, amp=amp)
    eager = [float(Trainer.train_one_step(m1, b, o1, s1, grad_clip=5.0)[0]) for b in batches]
    meta, d, m2, o2, s2 = _setup(dropout=0.1, amp=amp)
    run = CapturedTrainStep(m2, o2, s2, grad_clip=5.0, warmup=1)
    graph = [float(run(b)[0]) for b in batches]
    assert len(run.graphs) == 1
    assert eager == graph
    assert len(set(eager)) == len(eager)
    for (k, p1), p2 in zip(m1.state_dict().items(), m2.state_dict().values()):
        assert torch.equal(p1, p2), k
    # dropout masks differ between steps: the same batch twice gives two losses
    l_a = float(run(batches[0])[0])
    l_b = float(run(batches[0])[0])
    assert l_a != l_b


def test_nonfinite_grad_norm_skips_update_and_schedule():
    from espnet_amd.train.trainer import Trainer
    meta, d, m, opt, sched = _setup()
    batch = {k: torch.from_numpy(v) for k, v in section(d, "in0").items()}
    Trainer.train_one_step(m, batch, opt, sched, grad_clip=5.0)
    before = {k: v.clone() for k, v in m.state_dict().items() if "running" not in k and "num_batches" not in k}
    bad = dict(batch)
    bad["speech"] = batch["speech"].clone()
    bad["speech"][0, 3, 5] = float("nan")
    _, _, _, gn = Trainer.train_one_step(m, bad, opt, sched, grad_clip=5.0)
    assert not np.isfinite(float(gn))
    assert opt.step_count == 1
    for k, v in before.items():
        assert torch.equal(m.state_dict()[k], v), k
    assert float(m.arena.grad.abs().max()) == 0.0  # zero_grad still ran


def test_ctc_backward_fork_is_bit_exact_at_c3():
    """The CTC head's backward forked onto the auxiliary stream beside the decoder backward
    (hip_ops.OVERLAP_CTC_BWD) gives bit-identical losses and parameters to the serial order
    over several captured C3 steps (bf16, dropout on): no buffer is shared across the
    streams while both run."""
    import bench
    from espnet_amd import hip_ops as ops
    from espnet_amd.optim.adam import ArenaAdam
    from espnet_amd.schedulers.warmup_lr import WarmupLR
    from espnet_amd.train.graph import CapturedTrainStep

    cfg = bench.c3_config()
    host = bench.synthetic_batch(cfg, 1)
    runs = []
    saved = ops.OVERLAP_CTC_BWD
    try:
        for fork in (True, False):
            ops.OVERLAP_CTC_BWD = fork
            m = bench.build(cfg)
            m.prepare("cuda:0", amp=True, seed=1234)
            m.train()
            opt = ArenaAdam(m, lr=cfg["optim"]["lr"], weight_decay=cfg["optim"]["weight_decay"])
            sched = WarmupLR(opt, warmup_steps=cfg["warmup_steps"])
            batch = {k: v.to("cuda:0") for k, v in host.items()}
            step = CapturedTrainStep(m, opt, sched, grad_clip=5.0, warmup=2)
            losses = [float(step(batch, (cfg["T"], cfg["L"]))[0].item()) for _ in range(6)]
            torch.cuda.synchronize()
            runs.append((losses, m.arena.data.double().sum().item(), m.arena.data[:4096].clone().cpu()))
            del m, opt, sched, step
            torch.cuda.empty_cache()
    finally:
        ops.OVERLAP_CTC_BWD = saved
    assert runs[0][0] == runs[1][0]
    assert runs[0][1] == runs[1][1]
    assert torch.equal(runs[0][2], runs[1][2])


def test_three_specaug_steps_follow_reference_rng_stream():
    """Three eager training steps with SpecAug under one torch.manual_seed against the
    reference's own 3-step run (tests/golden/train3_specaug.npz): the host draws of step k+1
    (TimeWarp / masks) come after step k's MultiSequential draws (repeat.py:27), which the
    build replicates, so every step sees the reference's augmentation.  Tolerances: the
    HIP bicubic warp differs from ATen's by <= 5e-5 (tests/test_specaug.py)."""
    from test_model_build import build
    from espnet_amd.asr.specaug import SpecAug
    from espnet_amd.optim.adam import ArenaAdam
    from espnet_amd.schedulers.warmup_lr import WarmupLR
    from espnet_amd.train.trainer import Trainer
    meta, d = load("train3_specaug")
    cfg, _ = load(meta["cfg_name"])
    torch.manual_seed(0)
    m = build(cfg)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in section(d, "w").items()})
    m.specaug = SpecAug(**meta["specaug"])
    m.prepare("cuda:0", amp=False)
    m.train()
    opt = ArenaAdam(m, lr=meta["lr"], weight_decay=meta["weight_decay"])
    sched = WarmupLR(opt, warmup_steps=meta["warmup_steps"])
    torch.manual_seed(meta["seed"])
    for s in range(meta["steps"]):
        batch = {k: torch.from_numpy(v) for k, v in section(d, f"in{s}").items()}
        loss, _, _, _ = Trainer.train_one_step(m, batch, opt, sched, grad_clip=meta["grad_clip"])
        np.testing.assert_allclose(float(loss), d[f"out{s}.loss"], rtol=2e-5, atol=1e-4)
    sd = m.state_dict()
    for k, v in section(d, "w_after").items():
        tol = 1e-3 if k.endswith("depthwise_conv.bias") else 1e-4
        np.testing.assert_allclose(sd[k].cpu().float().numpy(), v, atol=tol, rtol=1e-4, err_msg=k)


@pytest.mark.parametrize("equal_lengths", [False, True])
def test_captured_specaug_steps_equal_eager(equal_lengths):
    """SpecAug steps captured as a hipGraph (draws made on the host before each replay into
    SpecAug's static device buffer, MultiSequential's draws before the replay too) give
    bit-identical losses and parameters to eager SpecAug steps under the same torch seed;
    with equal lengths this also checks that the captured per-utterance warp equals the
    reference's batch warp (time_warp.py:73-86)."""
    from test_model_build import build
    from espnet_amd.asr.specaug import SpecAug
    from espnet_amd.optim.adam import ArenaAdam
    from espnet_amd.schedulers.warmup_lr import WarmupLR
    from espnet_amd.train.graph import CapturedTrainStep
    from espnet_amd.train.trainer import Trainer
    meta, d = load("train3_specaug")
    cfg, _ = load(meta["cfg_name"])
    base = {k: torch.from_numpy(v) for k, v in section(d, "in0").items()}
    if equal_lengths:
        T = int(base["speech_lengths"].max())
        base["speech_lengths"] = torch.full_like(base["speech_lengths"], T)
    g = torch.Generator().manual_seed(3)
    batches = [dict(base, speech=torch.randn(base["speech"].shape, generator=g)) for _ in range(4)]

    def setup():
        torch.manual_seed(0)
        m = build(cfg)
        m.load_state_dict({k: torch.from_numpy(v) for k, v in section(d, "w").items()})
        m.specaug = SpecAug(**meta["specaug"])
        m.prepare("cuda:0", amp=True, seed=5)
        m.train()
        opt = ArenaAdam(m, lr=meta["lr"], weight_decay=meta["weight_decay"])
        return m, opt, WarmupLR(opt, warmup_steps=meta["warmup_steps"])

    m1, o1, s1 = setup()
    torch.manual_seed(99)
    eager = [float(Trainer.train_one_step(m1, b, o1, s1, grad_clip=5.0)[0]) for b in batches]
    rng_eager = torch.get_rng_state()
    m2, o2, s2 = setup()
    run = CapturedTrainStep(m2, o2, s2, grad_clip=5.0, warmup=1)
    torch.manual_seed(99)
    graph = [float(run(b)[0]) for b in batches]
    assert len(run.graphs) == 1
    assert eager == graph
    assert torch.equal(rng_eager, torch.get_rng_state())  # the same host draws, in the same order
    for (k, p1), p2 in zip(m1.state_dict().items(), m2.state_dict().values()):
        assert torch.equal(p1, p2), k


@pytest.mark.parametrize("amp", [False, True])
def test_ctc_backward_in_forward_matches_after(amp):
    """layers/losses.py CTC_BWD_IN_FWD: the CTC head's backward computed in the forward for an
    upstream gradient of 1 and scaled by the real one in the backward equals the head backward
    run after the decoder's (the same arithmetic up to where the scale enters: fp32 to 1e-6,
    bf16 to its rounding of the unscaled gradient), over two training steps."""
    from test_dp_capture_gpu import _batches, _setup
    from espnet_amd.layers import losses as Lo
    from espnet_amd.train.trainer import Trainer
    out = {}
    saved = Lo.CTC_BWD_IN_FWD
    try:
        for pre in (False, True):
            Lo.CTC_BWD_IN_FWD = pre
            d, m, opt, sched = _setup(amp=amp, dropout=0.1)
            losses = [float(Trainer.train_one_step(m, b, opt, sched, grad_clip=5.0)[0]) for b in _batches(d, 2)]
            torch.cuda.synchronize()
            out[pre] = (losses, m.arena.data.cpu().clone())
    finally:
        Lo.CTC_BWD_IN_FWD = saved
    np.testing.assert_allclose(out[True][0], out[False][0], rtol=1e-6 if not amp else 1e-4)
    w0, w1 = out[False][1].double(), out[True][1].double()
    tol = 1e-5 if not amp else 2e-3  # (two Adam steps amplify fp32 rounding: 1.6e-6 measured)
    assert float((w1 - w0).norm() / w0.norm()) < tol
