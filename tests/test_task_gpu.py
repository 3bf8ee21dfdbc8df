"""The training loop and the command-line entry on the MI355X.

* Trainer.train_one_epoch with accum_grad=2 against the reference's own
  Trainer.train_one_epoch (oracle/make_goldens.py capture_epoch: 4 batches, two backwards
  per update, clip + Adam + WarmupLR every 2nd batch): parameters after the epoch and the
  reporter's epoch aggregates (loss, loss_ctc, loss_att, acc, optim0_lr0) — the timers
  (iter_time, forward_time, backward_time, optim_step_time, train_time) must be reported,
  from the device phase stamps.
* ASRTask.main end-to-end (espnet2/tasks/abs_task.py:1026-1357 + trainer.py:162-470) on a
  rand_float / text_int corpus written to disk: YAML config + command-line flags, bf16 AMP,
  two epochs of captured steps, validation, checkpoint / epoch files / best links / n-best
  average, then --resume continuing to a third epoch.
"""
import json
import math

import numpy as np
import pytest
import torch

from goldens import load, section

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("captured", [False, True])
def test_train_one_epoch_accum_grad_matches_reference(captured):
    """accum_grad=2 epoch against the reference's own epoch golden; captured=True runs it through
    graph.CapturedTrainStep (warm-up 1): the micro-step graph is captured at batch 3 and the
    updating micro-step's graph at batch 4 (two graphs per shape, trainer.py:619-653)."""
    from test_model_build import build
    from espnet_amd.optim.adam import ArenaAdam
    from espnet_amd.schedulers.warmup_lr import WarmupLR
    from espnet_amd.train.reporter import Reporter
    from espnet_amd.train.trainer import Trainer, TrainerOptions

    meta, d = load("epoch_accum2")
    cfg, _ = load(meta["cfg_name"])
    torch.manual_seed(0)
    m = build(cfg)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in section(d, "w").items()})
    m.prepare("cuda:0", amp=False)
    opt = ArenaAdam(m, lr=meta["lr"], weight_decay=meta["weight_decay"])
    sched = WarmupLR(opt, warmup_steps=meta["warmup_steps"])
    batches = []
    for s in range(meta["n_batches"]):
        b = {k: torch.from_numpy(v) for k, v in section(d, f"in{s}").items()}
        batches.append(([f"u{s}_{i}" for i in range(len(b["speech"]))], b))
    opts = TrainerOptions(ngpu=1, resume=False, use_amp=False, train_dtype="float32", grad_noise=False,
                          accum_grad=meta["accum_grad"], grad_clip=meta["grad_clip"], grad_clip_type=2.0,
                          log_interval=None, no_forward_run=False, use_matplotlib=False, use_tensorboard=False,
                          use_wandb=False, output_dir="/tmp", max_epoch=1, seed=0, sharded_ddp=False,
                          patience=None, keep_nbest_models=[1], nbest_averaging_interval=0,
                          early_stopping_criterion=("valid", "loss", "min"),
                          best_model_criterion=[("train", "loss", "min")], val_scheduler_criterion=("valid", "loss"),
                          unused_parameters=False, wandb_model_log_interval=-1, create_graph_in_tensorboard=False)
    runner = None
    if captured:
        from espnet_amd.train.graph import CapturedTrainStep
        runner = CapturedTrainStep(m, opt, sched, grad_clip=meta["grad_clip"], warmup=1,
                                   accum_grad=meta["accum_grad"])
    rep = Reporter()
    rep.set_epoch(1)
    with rep.observe("train") as sub:
        invalid = Trainer.train_one_epoch(m, iter(batches), [opt], [sched], reporter=sub, options=opts,
                                          step_runner=runner)
    if captured:
        assert runner.mode == "graph" and [c for c, _ in runner.captures] == [3, 4], runner.captures
    torch.cuda.synchronize()
    assert invalid == bool(d["all_invalid"])
    st = rep.stats[1]["train"]
    assert st["total_count"] == int(d["total_count"])
    for k in json.loads(str(d["stats_keys"])):
        np.testing.assert_allclose(st[k], float(d["stat." + k]), rtol=2e-6, atol=1e-5, err_msg=k)
    for k in json.loads(str(d["time_keys"])):
        assert k in st and math.isfinite(st[k]) and st[k] >= 0, k
    assert 0 < st["forward_time"] < 1.0 and 0 < st["backward_time"] < 1.0 and 0 < st["optim_step_time"] < 1.0
    sd = m.state_dict()
    for k, v in section(d, "w_after").items():
        tol = 6e-4 if k.endswith("depthwise_conv.bias") else 5e-5  # tests/test_trainer_gpu.py
        np.testing.assert_allclose(sd[k].cpu().float().numpy(), v, atol=tol, rtol=1e-5, err_msg=k)


def test_train_one_epoch_all_invalid_follows_skipped_updates():
    """trainer.py:662-681: a step whose grad norm is non-finite skips the update and registers
    no optim_step_time; an epoch whose every update was skipped returns
    all_steps_are_invalid=True (run() then stops).  The skip is decided on the device
    (ArenaAdam): the epoch reads the applied-update count once at its end."""
    from test_model_build import build
    from espnet_amd.optim.adam import ArenaAdam
    from espnet_amd.train.reporter import Reporter
    from espnet_amd.train.trainer import Trainer, TrainerOptions

    cfg, d = load("tiny_hybrid")
    torch.manual_seed(0)
    m = build(cfg)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in section(d, "w").items()})
    m.prepare("cuda:0", amp=False)
    opt = ArenaAdam(m, lr=1e-3)
    inp = {k: torch.from_numpy(v) for k, v in section(d, "in").items()}
    bad = dict(inp, speech=inp["speech"].clone())
    bad["speech"][0, 0, 0] = float("nan")
    opts = TrainerOptions(ngpu=1, resume=False, use_amp=False, train_dtype="float32", grad_noise=False,
                          accum_grad=1, grad_clip=5.0, grad_clip_type=2.0, log_interval=None,
                          no_forward_run=False, use_matplotlib=False, use_tensorboard=False, use_wandb=False,
                          output_dir="/tmp", max_epoch=1, seed=0, sharded_ddp=False, patience=None,
                          keep_nbest_models=[1], nbest_averaging_interval=0,
                          early_stopping_criterion=("valid", "loss", "min"),
                          best_model_criterion=[("train", "loss", "min")], val_scheduler_criterion=("valid", "loss"),
                          unused_parameters=False, wandb_model_log_interval=-1, create_graph_in_tensorboard=False)
    ids = [f"u{i}" for i in range(len(inp["speech"]))]
    before = m.state_dict()["ctc.ctc_lo.weight"].clone()
    rep = Reporter()
    rep.set_epoch(1)
    with rep.observe("train") as sub:
        invalid = Trainer.train_one_epoch(m, iter([(ids, bad), (ids, bad)]), [opt], [], reporter=sub, options=opts)
    assert invalid is True
    assert opt.step_count == 0
    assert torch.equal(m.state_dict()["ctc.ctc_lo.weight"], before)
    st = rep.stats[1]["train"]
    assert not math.isfinite(st.get("optim_step_time", float("nan")))
    rep.set_epoch(2)
    with rep.observe("train") as sub:
        invalid = Trainer.train_one_epoch(m, iter([(ids, bad), (ids, inp), (ids, bad)]), [opt], [], reporter=sub,
                                          options=opts)
    assert invalid is False
    assert opt.step_count == 1
    st = rep.stats[2]["train"]
    assert 0 < st["optim_step_time"] < 1.0  # the mean over the one applied update


def _corpus(tmp_path, n, T=(60, 140), L=(3, 12), V=30, seed=0):
    rng = np.random.RandomState(seed)
    shp, txt, tshp = [], [], []
    for i in range(n):
        t = int(rng.randint(*T))
        l_ = int(rng.randint(*L))
        shp.append(f"utt{i:03d} {t},80")
        txt.append(f"utt{i:03d} " + " ".join(str(int(x)) for x in rng.randint(2, V - 1, size=l_)))
        tshp.append(f"utt{i:03d} {l_}")
    for name, lines in (("speech_shape", shp), ("text", txt), ("text_shape", tshp)):
        (tmp_path / name).write_text("\n".join(lines) + "\n")
    return tmp_path


def test_asr_task_main_end_to_end_and_resume(tmp_path):
    import yaml
    from espnet_amd.tasks.asr import ASRTask

    (tmp_path / "tr").mkdir()
    (tmp_path / "dv").mkdir()
    tr = _corpus(tmp_path / "tr", 24)
    dv = _corpus(tmp_path / "dv", 6, seed=1)
    V = 30
    (tmp_path / "tokens.txt").write_text("\n".join(["<blank>", "<unk>"] + [f"c{i}" for i in range(V - 3)]
                                                   + ["<sos/eos>"]) + "\n")
    conf = dict(encoder="transformer",
                encoder_conf=dict(output_size=64, attention_heads=4, linear_units=256, num_blocks=2),
                decoder="transformer", decoder_conf=dict(attention_heads=4, linear_units=256, num_blocks=2),
                model_conf=dict(ctc_weight=0.3, lsm_weight=0.1, length_normalized_loss=False),
                optim="adam", optim_conf=dict(lr=0.002), scheduler="warmuplr", scheduler_conf=dict(warmup_steps=10),
                batch_type="sorted", batch_size=4, max_epoch=2, use_amp=True, num_workers=0,
                best_model_criterion=[["valid", "loss", "min"], ["train", "acc", "max"]], keep_nbest_models=[1, 2],
                use_preprocessor=False)
    (tmp_path / "c.yaml").write_text(yaml.safe_dump(conf))
    out = tmp_path / "exp"
    cmd = ["--config", str(tmp_path / "c.yaml"), "--output_dir", str(out), "--ngpu", "1",
           "--token_list", str(tmp_path / "tokens.txt"), "--input_size", "80",
           "--train_data_path_and_name_and_type", f"{tr}/speech_shape,speech,rand_float",
           "--train_data_path_and_name_and_type", f"{tr}/text,text,text_int",
           "--train_shape_file", f"{tr}/speech_shape",
           "--valid_data_path_and_name_and_type", f"{dv}/speech_shape,speech,rand_float",
           "--valid_data_path_and_name_and_type", f"{dv}/text,text,text_int",
           "--valid_shape_file", f"{dv}/speech_shape"]
    ASRTask.main(cmd=cmd)
    files = {p.name for p in out.iterdir()}
    assert {"config.yaml", "checkpoint.pth", "latest.pth", "valid.loss.best.pth", "valid.loss.ave.pth",
            "train.acc.ave.pth"} <= files, files
    assert any(f.endswith("epoch.pth") for f in files)
    ck = torch.load(out / "checkpoint.pth", map_location="cpu", weights_only=True)
    assert ck["reporter"]["epoch"] == 2
    st = ck["reporter"]["stats"][2]["train"]
    for k in ("loss", "loss_ctc", "loss_att", "acc", "iter_time", "forward_time", "backward_time",
              "optim_step_time", "train_time", "optim0_lr0"):
        assert k in st and math.isfinite(st[k]), (k, st.get(k))
    assert st["total_count"] == 2 * 6
    assert "loss" in ck["reporter"]["stats"][2]["valid"]
    assert yaml.safe_load((out / "config.yaml").read_text())["encoder"] == "transformer"
    # resume: a third epoch continues from the checkpoint
    ASRTask.main(cmd=cmd + ["--resume", "true", "--max_epoch", "3"])
    ck3 = torch.load(out / "checkpoint.pth", map_location="cpu", weights_only=True)
    assert ck3["reporter"]["epoch"] == 3
    assert ck3["reporter"]["stats"][3]["train"]["total_count"] == 3 * 6
    assert int(ck3["optimizers"][0]["state"][0]["step"]) == 18


def test_asr_task_main_two_spawned_workers_match_one_process(tmp_path):
    """The recipe launch of a DP job (abs_task.py:1041-1094): ASRTask.main --ngpu 2
    --multiprocessing_distributed true spawns one main_worker per rank; with --dist_backend
    gloo both workers share cuda:0 (DistributedOption.device_index), so the multi-worker entry
    point runs on the one-GPU box.  Each rank trains on batch[rank::2] of every global batch
    with the gradient all-reduce and the DP loss weighting (trainer.py:604-619), so with no
    dropout, an encoder without BatchNorm (per-replica statistics) and utterances of one
    length the two-worker job trains the same model as one process on the whole batches:
    rank 0's checkpoint equals the single-process run's (fp32; only reduction order differs).
    (Equal lengths: the reference's Conv2dSubsampling lengths come from slicing the PADDED
    mask, x_mask[:, :, :-2:2][:, :, :-2:2] (subsampling.py:91), so a padded utterance keeps
    one more CTC frame than the same utterance unpadded — a rank's shard, padded to its own
    maximum, is not the same computation as the whole batch; the oracle shows the same split.)
    Adam's eps is 1 here: the first updates are then ~lr*g instead of ~lr*sign(g), whose sign
    flips on near-zero gradient entries would turn reduction-order noise into lr-sized
    parameter differences."""
    import yaml
    from espnet_amd.tasks.asr import ASRTask

    (tmp_path / "tr").mkdir()
    (tmp_path / "dv").mkdir()
    tr = _corpus(tmp_path / "tr", 16, T=(120, 121))
    dv = _corpus(tmp_path / "dv", 4, T=(120, 121), seed=1)
    # fixed features (npy): rand_float draws from each process's own numpy stream
    for d_, seed in ((tr, 3), (dv, 4)):
        rng = np.random.RandomState(seed)
        lines = []
        for ln in (d_ / "speech_shape").read_text().split("\n"):
            if ln:
                utt, shp = ln.split()
                f = d_ / f"{utt}.npy"
                np.save(f, rng.randn(*[int(x) for x in shp.split(",")]).astype(np.float32))
                lines.append(f"{utt} {f}")
        (d_ / "feats.scp").write_text("\n".join(lines) + "\n")
    V = 30
    (tmp_path / "tokens.txt").write_text("\n".join(["<blank>", "<unk>"] + [f"c{i}" for i in range(V - 3)]
                                                   + ["<sos/eos>"]) + "\n")
    conf = dict(encoder="transformer",
                encoder_conf=dict(output_size=64, attention_heads=4, linear_units=256, num_blocks=2,
                                  dropout_rate=0.0, positional_dropout_rate=0.0, attention_dropout_rate=0.0),
                decoder="transformer",
                decoder_conf=dict(attention_heads=4, linear_units=256, num_blocks=2, dropout_rate=0.0,
                                  positional_dropout_rate=0.0, self_attention_dropout_rate=0.0,
                                  src_attention_dropout_rate=0.0),
                model_conf=dict(ctc_weight=0.3, lsm_weight=0.1, length_normalized_loss=False),
                optim="adam", optim_conf=dict(lr=0.002, eps=1.0), scheduler="warmuplr",
                scheduler_conf=dict(warmup_steps=10), batch_type="sorted", batch_size=4, max_epoch=1, use_amp=False,
                num_workers=0, best_model_criterion=[["valid", "loss", "min"]], keep_nbest_models=1,
                use_preprocessor=False)
    (tmp_path / "c.yaml").write_text(yaml.safe_dump(conf))

    def cmd(out, ngpu):
        return ["--config", str(tmp_path / "c.yaml"), "--output_dir", str(out), "--ngpu", str(ngpu),
                "--token_list", str(tmp_path / "tokens.txt"), "--input_size", "80",
                "--train_data_path_and_name_and_type", f"{tr}/feats.scp,speech,npy",
                "--train_data_path_and_name_and_type", f"{tr}/text,text,text_int",
                "--train_shape_file", f"{tr}/speech_shape",
                "--valid_data_path_and_name_and_type", f"{dv}/feats.scp,speech,npy",
                "--valid_data_path_and_name_and_type", f"{dv}/text,text,text_int",
                "--valid_shape_file", f"{dv}/speech_shape"]

    ASRTask.main(cmd=cmd(tmp_path / "one", 1))
    ASRTask.main(cmd=cmd(tmp_path / "two", 2) + ["--dist_backend", "gloo", "--multiprocessing_distributed", "true"])
    c1 = torch.load(tmp_path / "one" / "checkpoint.pth", map_location="cpu", weights_only=True)
    c2 = torch.load(tmp_path / "two" / "checkpoint.pth", map_location="cpu", weights_only=True)
    assert c1["reporter"]["epoch"] == c2["reporter"]["epoch"] == 1
    s1, s2 = c1["reporter"]["stats"][1]["train"], c2["reporter"]["stats"][1]["train"]
    assert s2["total_count"] == s1["total_count"] == 4  # 4 global batches, one update each
    # (acc is a per-rank token ratio averaged with utterance weights, as in the reference: not
    # the single-process ratio)
    for k in ("loss", "loss_ctc", "loss_att"):
        np.testing.assert_allclose(s2[k], s1[k], rtol=1e-5, atol=1e-5, err_msg=k)
    assert int(c2["optimizers"][0]["state"][0]["step"]) == 4
    for k, v in c1["model"].items():
        np.testing.assert_allclose(c2["model"][k].float().numpy(), v.float().numpy(), atol=1e-5, rtol=1e-4,
                                   err_msg=k)
    v1, v2 = c1["reporter"]["stats"][1]["valid"], c2["reporter"]["stats"][1]["valid"]
    np.testing.assert_allclose(v2["loss"], v1["loss"], rtol=1e-5)
