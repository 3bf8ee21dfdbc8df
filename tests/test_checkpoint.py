"""Checkpoint / model-file interop (espnet2/train/trainer.py:133-159,
348-369, main_funcs/average_nbest_models.py): n-best averaging against the reference's own
output (tests/golden/avg_nbest.npz), and on the GPU a save -> resume round trip that must
continue the reference's 2-step Adam + WarmupLR run (tests/golden/train2.npz), plus our
checkpoint resumed by a plain torch.optim.Adam (the reference's optimizer) on the oracle."""
import json

import numpy as np
import pytest
import torch

from goldens import load, section


def test_average_nbest_models_matches_reference(tmp_path):
    from espnet_amd.train.checkpoint import EpochReporter, average_nbest_models
    cfg, d = load("avg_nbest")
    rep = EpochReporter()
    for e in (1, 2, 3, 4):
        sd = {k: torch.from_numpy(d[f"epoch{e}.{k}"]) for k in ("w", "b", "bn.num_batches_tracked")}
        torch.save(sd, tmp_path / f"{e}epoch.pth")
        rep.set_epoch(e)
        rep.register("valid", {"loss": cfg["losses"][str(e)], "acc": cfg["accs"][str(e)]})
    average_nbest_models(tmp_path, rep, [("valid", "loss", "min"), ("valid", "acc", "max")], [1, 2, 3])
    files = sorted(p.name for p in tmp_path.iterdir())
    assert files == cfg["files"]
    links = {p.name: str(p.readlink()) for p in tmp_path.iterdir() if p.is_symlink()}
    assert links == cfg["links"]
    for f in files:
        if "ave" in f and not (tmp_path / f).is_symlink():
            sd = torch.load(tmp_path / f, weights_only=True)
            for k, v in sd.items():
                ref = d[f"{f}.{k}"]
                assert v.dtype == torch.from_numpy(ref).dtype, (f, k)
                np.testing.assert_array_equal(v.numpy(), ref, err_msg=f"{f}.{k}")


def test_reporter_state_roundtrip():
    from espnet_amd.train.checkpoint import EpochReporter
    r = EpochReporter()
    for e, v in ((1, 2.0), (2, 1.0), (3, 3.0)):
        r.set_epoch(e)
        r.register("valid", {"loss": v})
    assert r.get_best_epoch("valid", "loss", "min") == 2
    assert r.sort_epochs("valid", "loss", "max") == [3, 1, 2]
    r2 = EpochReporter()
    r2.load_state_dict(r.state_dict())
    assert r2.stats == r.stats and r2.get_epoch() == 3


@pytest.mark.gpu
def test_checkpoint_resume_continues_reference_run(tmp_path):
    from oracle.asr_oracle import OracleASR, OracleTrainer
    from test_model_build import build
    from espnet_amd.optim.adam import ArenaAdam
    from espnet_amd.schedulers.warmup_lr import WarmupLR
    from espnet_amd.train.checkpoint import EpochReporter, resume, save_checkpoint, save_epoch_model
    from espnet_amd.train.trainer import Trainer

    tc, d = load("train2")
    cfg, _ = load(tc["cfg_name"])
    w0 = {k: torch.from_numpy(v) for k, v in section(d, "w").items()}

    def fresh():
        torch.manual_seed(0)
        m = build(cfg)
        m.load_state_dict(w0)
        m.prepare("cuda", amp=False)
        m.train()
        opt = ArenaAdam(m, lr=tc["lr"], weight_decay=tc["weight_decay"])
        return m, opt, WarmupLR(opt, warmup_steps=tc["warmup_steps"])

    batch = lambda s: {k: torch.from_numpy(v) for k, v in section(d, f"in{s}").items()}
    m, opt, sched = fresh()
    Trainer.train_one_step(m, batch(0), opt, sched, grad_clip=tc["grad_clip"])
    rep = EpochReporter(epoch=1)
    rep.register("train", {"loss": 1.0})
    save_checkpoint(tmp_path, m, rep, [opt], [sched])
    save_epoch_model(tmp_path, m, 1)
    assert (tmp_path / "latest.pth").readlink().name == "1epoch.pth"

    # 1) our own resume: a fresh model/optimizer/scheduler continues to the reference's step 2
    m2, opt2, sched2 = fresh()
    rep2 = EpochReporter()
    resume(tmp_path / "checkpoint.pth", m2, rep2, [opt2], [sched2], ngpu=1)
    assert rep2.state_dict() == rep.state_dict()
    Trainer.train_one_step(m2, batch(1), opt2, sched2, grad_clip=tc["grad_clip"])
    torch.cuda.synchronize()
    sd = m2.state_dict()
    # tolerances of tests/test_trainer_gpu.py (Adam's sign-like update of near-zero gradient
    # elements amplifies f32 rounding; the BN-fed depthwise bias most)
    tol = lambda k: 6e-4 if k.endswith("depthwise_conv.bias") else 5e-5  # noqa: E731
    for k, v in section(d, "w_after").items():
        np.testing.assert_allclose(sd[k].cpu().numpy(), v, atol=tol(k), rtol=1e-5, err_msg=k)

    # 2) the reference's optimizer (torch.optim.Adam on the CPU oracle) resumes our checkpoint
    ck = torch.load(tmp_path / "checkpoint.pth", map_location="cpu", weights_only=True)
    assert set(ck) == {"model", "reporter", "optimizers", "schedulers", "scaler"}
    ora = OracleASR(cfg, {k: v.clone() for k, v in ck["model"].items()})
    tr = OracleTrainer(ora, tc["lr"], tc["weight_decay"], tc["warmup_steps"], tc["grad_clip"])
    tr.opt.load_state_dict(ck["optimizers"][0])
    tr.step_num = ck["schedulers"][0]["last_epoch"] + 1
    for g in tr.opt.param_groups:
        g["lr"] = tc["lr"] * tc["warmup_steps"] ** 0.5 * min(tr.step_num ** -0.5,
                                                             tr.step_num * tc["warmup_steps"] ** -1.5)
    tr.step(batch(1))
    for k, v in section(d, "w_after").items():
        if k in ora.params:
            np.testing.assert_allclose(ora.params[k].detach().numpy(), v, atol=tol(k), rtol=1e-5, err_msg=k)


@pytest.mark.gpu
def test_amp_resume_into_prepared_model_uses_loaded_weights(tmp_path):
    """Under AMP the GEMMs read the bf16 weight shadow: loading weights into an already
    prepared model (resume, n-best averaged models) must refresh it.  The first step after
    resume() into a prepared, randomly initialised model must equal the first step of a
    model that loaded the same checkpoint before prepare()."""
    from test_model_build import build
    from espnet_amd.optim.adam import ArenaAdam
    from espnet_amd.schedulers.warmup_lr import WarmupLR
    from espnet_amd.train.checkpoint import EpochReporter, resume, save_checkpoint
    from espnet_amd.train.trainer import Trainer

    tc, d = load("train2")
    cfg, _ = load(tc["cfg_name"])
    w0 = {k: torch.from_numpy(v) for k, v in section(d, "w").items()}
    batch = lambda s: {k: torch.from_numpy(v) for k, v in section(d, f"in{s}").items()}  # noqa: E731

    def opt_sched(m):
        opt = ArenaAdam(m, lr=tc["lr"], weight_decay=tc["weight_decay"])
        return opt, WarmupLR(opt, warmup_steps=tc["warmup_steps"])

    torch.manual_seed(0)
    m = build(cfg)
    m.load_state_dict(w0)
    m.prepare("cuda", amp=True)
    m.train()
    opt, sched = opt_sched(m)
    Trainer.train_one_step(m, batch(0), opt, sched, grad_clip=tc["grad_clip"])
    save_checkpoint(tmp_path, m, EpochReporter(epoch=1), [opt], [sched])

    # resumed into a prepared model whose arena (and bf16 shadow) hold a different init
    torch.manual_seed(123)
    m2 = build(cfg)
    m2.prepare("cuda", amp=True)
    m2.train()
    opt2, sched2 = opt_sched(m2)
    resume(tmp_path / "checkpoint.pth", m2, EpochReporter(), [opt2], [sched2], ngpu=1)
    loss2, _, _, _ = Trainer.train_one_step(m2, batch(1), opt2, sched2, grad_clip=tc["grad_clip"])

    # reference: the checkpoint's weights loaded before prepare()
    ck = torch.load(tmp_path / "checkpoint.pth", map_location="cpu", weights_only=True)
    m3 = build(cfg)
    m3.load_state_dict(ck["model"])
    m3.prepare("cuda", amp=True)
    m3.train()
    opt3, sched3 = opt_sched(m3)
    opt3.load_state_dict(ck["optimizers"][0])
    sched3.load_state_dict(ck["schedulers"][0])
    loss3, _, _, _ = Trainer.train_one_step(m3, batch(1), opt3, sched3, grad_clip=tc["grad_clip"])
    torch.cuda.synchronize()
    np.testing.assert_allclose(loss2.item(), loss3.item(), rtol=1e-6)
    for k, v in m3.state_dict().items():
        np.testing.assert_allclose(m2.state_dict()[k].cpu().numpy(), v.cpu().numpy(), atol=1e-6, rtol=1e-6,
                                   err_msg=k)
    # eval forward of an averaged / loaded model on a prepared AMP model, same check
    m2.eval()
    m3.eval()
    m2.load_state_dict(w0)
    m3.load_state_dict(w0)
    l2, _, _ = m2(**batch(0))
    l3, _, _ = m3(**batch(0))
    np.testing.assert_allclose(l2.item(), l3.item(), rtol=1e-6)


@pytest.mark.gpu
def test_amp_submodule_load_refreshes_shadow():
    """Loading into a submodule of a prepared AMP model (model.encoder.load_state_dict, as the
    reference's init_param / load_pretrained_model do) refreshes the bf16 weight shadow the
    GEMMs read; a whole-model load refreshes it once."""
    from test_model_build import build

    tc, d = load("train2")
    cfg, _ = load(tc["cfg_name"])
    w0 = {k: torch.from_numpy(v) for k, v in section(d, "w").items()}
    torch.manual_seed(7)
    m = build(cfg)
    m.prepare("cuda", amp=True)
    calls = []
    real = m.arena.refresh_shadow
    m.arena.refresh_shadow = lambda: (calls.append(1), real())[1]
    enc = {k[len("encoder."):]: v for k, v in w0.items() if k.startswith("encoder.")}
    m.encoder.load_state_dict(enc)
    assert len(calls) == 1
    torch.cuda.synchronize()
    assert torch.equal(m.arena.shadow, m.arena.data.to(torch.bfloat16))
    m.load_state_dict(w0)
    assert len(calls) == 2  # once for the whole-model load, not once per submodule
    torch.cuda.synchronize()
    assert torch.equal(m.arena.shadow, m.arena.data.to(torch.bfloat16))
