"""Capture golden vectors by running the REFERENCE implementation (this container only).

TEST INFRASTRUCTURE — never imported by the product package.

The reference (DavidLBick/espnet-1 at /root/reference) is pure Python over PyTorch ATen
(SURVEY.md §2, §8c).  It imports here with the import-only stubs in `oracle/shim/`
(typeguard, humanfriendly, librosa, torch_complex, numba) and
PYTHONDONTWRITEBYTECODE so nothing is written into the reference tree.  The ASRTask
entry point itself does not import (hydra is absent), so models are built from the
module classes exactly as `espnet2/tasks/asr.py:476-602` (build_model) does.

Every fixture stores weights + inputs + outputs (+ grads) as float32/int64 arrays in a
compressed .npz under tests/golden/.  The weights are stored, not regenerated, so the
fixtures do not depend on torch's RNG stream.

Run:  PYTHONDONTWRITEBYTECODE=1 python -B oracle/make_goldens.py
"""
from __future__ import annotations

import json
import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = os.environ.get("ESPNET_REFERENCE", "/root/reference")
OUT = os.path.join(REPO, "tests", "golden")
sys.path[:0] = [os.path.join(HERE, "shim"), REF]

import numpy as np  # noqa: E402
import torch  # noqa: E402

torch.set_num_threads(4)


# --------------------------------------------------------------------------------------
# model builders (mirror espnet2/tasks/asr.py:476-602 for frontend=None, input_size=F)
# --------------------------------------------------------------------------------------
def token_list(V):
    return ["<blank>", "<unk>"] + [f"t{i}" for i in range(V - 3)] + ["<sos/eos>"]


def build_reference_model(cfg):
    from espnet2.asr.ctc import CTC
    from espnet2.asr.decoder.transformer_decoder import TransformerDecoder
    from espnet2.asr.encoder.conformer_encoder import ConformerEncoder
    from espnet2.asr.encoder.transformer_encoder import TransformerEncoder
    from espnet2.asr.espnet_model import ESPnetASRModel
    from espnet2.layers.utterance_mvn import UtteranceMVN

    V = cfg["vocab_size"]
    enc_cls = {"conformer": ConformerEncoder, "transformer": TransformerEncoder}[cfg["encoder"]]
    encoder = enc_cls(input_size=cfg["input_size"], **cfg["encoder_conf"])
    decoder = None
    if cfg.get("decoder"):
        decoder = TransformerDecoder(
            vocab_size=V, encoder_output_size=encoder.output_size(), **cfg["decoder_conf"]
        )
    ctc = CTC(odim=V, encoder_output_size=encoder.output_size(), **cfg.get("ctc_conf", {}))
    model = ESPnetASRModel(
        vocab_size=V,
        token_list=token_list(V),
        frontend=None,
        specaug=None,
        normalize=UtteranceMVN(),
        preencoder=None,
        encoder=encoder,
        postencoder=None,
        decoder=decoder,
        ctc=ctc,
        joint_network=None,
        **cfg["model_conf"],
    )
    return model


def perturb_norms(model, gen):
    """Make LayerNorm/BatchNorm affine params and BN running stats non-trivial so that
    the goldens discriminate gamma/beta/statistics bugs (defaults are 1/0)."""
    with torch.no_grad():
        for name, p in model.named_parameters():
            if "norm" in name:
                p.add_(0.1 * torch.randn(p.shape, generator=gen))
        for name, b in model.named_buffers():
            if name.endswith("running_mean"):
                b.copy_(0.1 * torch.randn(b.shape, generator=gen))
            elif name.endswith("running_var"):
                b.copy_(1.0 + 0.2 * torch.rand(b.shape, generator=gen))


def make_batch(cfg, gen):
    B = len(cfg["speech_lengths"])
    T = max(cfg["speech_lengths"])
    F = cfg["input_size"]
    V = cfg["vocab_size"]
    speech = torch.zeros(B, T, F)
    for b, t in enumerate(cfg["speech_lengths"]):
        speech[b, :t] = torch.randn(t, F, generator=gen)
    L = max(cfg["text_lengths"])
    text = torch.full((B, L), -1, dtype=torch.long)
    for b, l in enumerate(cfg["text_lengths"]):
        text[b, :l] = torch.randint(2, V - 1, (l,), generator=gen)
    return dict(
        speech=speech,
        speech_lengths=torch.tensor(cfg["speech_lengths"], dtype=torch.long),
        text=text,
        text_lengths=torch.tensor(cfg["text_lengths"], dtype=torch.long),
    )


def np32(t):
    t = t.detach().cpu()
    if t.dtype in (torch.float64, torch.float16, torch.bfloat16):
        t = t.float()
    return t.numpy().copy()  # a snapshot: buffers (BN running stats) are updated in place later


# --------------------------------------------------------------------------------------
# configs
# --------------------------------------------------------------------------------------
def conformer_conf(d, h, ff, nb, k=31, drop=0.0):
    return dict(
        output_size=d, attention_heads=h, linear_units=ff, num_blocks=nb,
        dropout_rate=drop, positional_dropout_rate=drop, attention_dropout_rate=drop,
        input_layer="conv2d", normalize_before=True, macaron_style=True,
        rel_pos_type="latest", pos_enc_layer_type="rel_pos",
        selfattention_layer_type="rel_selfattn", activation_type="swish",
        use_cnn_module=True, cnn_module_kernel=k,
    )


def decoder_conf(h, ff, nb, drop=0.0):
    return dict(
        attention_heads=h, linear_units=ff, num_blocks=nb, dropout_rate=drop,
        positional_dropout_rate=drop, self_attention_dropout_rate=drop,
        src_attention_dropout_rate=drop,
    )


CONFIGS = {
    # 2-block conformer + 2-block decoder, hybrid 0.3/0.7, lsm 0.1, ragged lengths
    "tiny_hybrid": dict(
        encoder="conformer", input_size=80, vocab_size=50,
        encoder_conf=conformer_conf(64, 4, 128, 2, k=15),
        decoder="transformer", decoder_conf=decoder_conf(4, 128, 2),
        model_conf=dict(ctc_weight=0.3, lsm_weight=0.1, length_normalized_loss=False),
        speech_lengths=[120, 97, 64, 33], text_lengths=[12, 9, 7, 3],
    ),
    # CTC-only (ctc_weight=1.0 -> decoder dropped), C2-style, kernel 31 > T'
    "tiny_ctc": dict(
        encoder="conformer", input_size=80, vocab_size=40,
        encoder_conf=conformer_conf(64, 4, 256, 2, k=31),
        decoder="transformer", decoder_conf=decoder_conf(4, 128, 1),
        model_conf=dict(ctc_weight=1.0, lsm_weight=0.0, length_normalized_loss=False),
        speech_lengths=[100, 100, 81], text_lengths=[10, 4, 8],
    ),
    # BASELINE.json configs[0] (C1): Transformer-tiny (2x64 encoder/decoder), mini_an4-shaped
    # batch of 2 (utterance lengths from the 8 mini_an4 recordings), V=30 characters
    "c1_tiny": dict(
        encoder="transformer", input_size=80, vocab_size=30,
        encoder_conf=dict(output_size=64, attention_heads=4, linear_units=256, num_blocks=2,
                          dropout_rate=0.0, positional_dropout_rate=0.0, attention_dropout_rate=0.0,
                          input_layer="conv2d", normalize_before=True),
        decoder="transformer", decoder_conf=decoder_conf(4, 256, 2),
        model_conf=dict(ctc_weight=0.3, lsm_weight=0.1, length_normalized_loss=False),
        speech_lengths=[290, 220], text_lengths=[14, 9],
    ),
    # realistic widths (d=256, h=4, ff=1024, d_k=64), one block each, equal lengths
    "medium_hybrid": dict(
        encoder="conformer", input_size=80, vocab_size=300,
        encoder_conf=conformer_conf(256, 4, 1024, 1, k=31),
        decoder="transformer", decoder_conf=decoder_conf(4, 1024, 1),
        model_conf=dict(ctc_weight=0.3, lsm_weight=0.1, length_normalized_loss=False),
        speech_lengths=[200, 200], text_lengths=[15, 15],
    ),
}


def capture_model(name, cfg, seed=0, light=False):
    torch.manual_seed(seed)
    model = build_reference_model(cfg)
    gen = torch.Generator().manual_seed(1000 + seed)
    perturb_norms(model, gen)
    batch = make_batch(cfg, torch.Generator().manual_seed(1))
    model.train()
    sd0 = {k: v.clone() for k, v in model.state_dict().items()}

    mids = {}
    hooks = []

    def keep(key):
        def fn(mod, inp, out):
            x = out
            if isinstance(x, tuple):
                x = x[0]
            if isinstance(x, tuple):
                mids[key + ".pos"] = np32(out[0][1])
                x = x[0]
            mids[key] = np32(x)

        return fn

    hooks.append(model.encoder.embed.register_forward_hook(keep("embed")))
    for i, layer in enumerate(model.encoder.encoders):
        hooks.append(layer.register_forward_hook(keep(f"enc{i}")))
    enc_out = {}

    def enc_hook(mod, inp, out):
        enc_out["x"], enc_out["lens"] = out[0], out[1]

    hooks.append(model.encoder.register_forward_hook(enc_hook))
    dec_out = {}
    if model.decoder is not None:
        def dec_hook(mod, inp, out):
            dec_out["x"] = out[0]

        hooks.append(model.decoder.register_forward_hook(dec_hook))

    inputs = {k: v.clone() for k, v in batch.items()}
    loss, stats, weight = model(**batch)
    loss.backward()
    for h in hooks:
        h.remove()

    rec = {"cfg": np.array(json.dumps({k: v for k, v in cfg.items()}))}
    for k, v in sd0.items():
        rec["w." + k] = np32(v)
    for k, v in inputs.items():
        rec["in." + k] = v.numpy()
    rec["out.loss"] = np32(loss)
    for k, v in stats.items():
        if v is not None:
            rec["stat." + k] = np32(v)
    rec["out.weight"] = weight.numpy()
    rec["out.encoder_out"] = np32(enc_out["x"])
    rec["out.encoder_out_lens"] = enc_out["lens"].numpy()
    with torch.no_grad():
        rec["out.ctc_argmax"] = model.ctc.argmax(enc_out["x"]).numpy()
        rec["out.ctc_logits"] = np32(model.ctc.ctc_lo(enc_out["x"]))
    if dec_out:
        rec["out.decoder_out"] = np32(dec_out["x"])
    for k, v in mids.items():
        rec["mid." + k] = v
    for k, p in model.named_parameters():
        if p.grad is None:
            continue
        if light and p.numel() > 4096:
            # keep the fixture small: norm, sum and a 256-element head of big grads
            g = p.grad.detach().double()
            rec["gn." + k] = np.array(g.norm().item())
            rec["gs." + k] = np.array(g.sum().item())
            rec["gh." + k] = np32(p.grad.reshape(-1)[:256])
        else:
            rec["g." + k] = np32(p.grad)
    if light:
        rec = {k: v for k, v in rec.items() if not k.startswith("mid.enc")}
    for k, v in model.state_dict().items():
        if "running" in k or "num_batches" in k:
            rec["buf_after." + k] = np32(v)
    path = os.path.join(OUT, f"{name}.npz")
    np.savez_compressed(path, **rec)
    print(f"{name}: loss={loss.item():.6f} stats={ {k: (float(v) if v is not None else None) for k, v in stats.items()} } -> {path} ({os.path.getsize(path)/1e6:.2f} MB)")


def capture_train_steps(name="train2", cfg_name="tiny_hybrid", steps=2):
    """Two Trainer steps (trainer.py:604-701 semantics, single process):
    loss.backward -> clip_grad_norm_(5.0) -> Adam(lr, wd) step -> WarmupLR step -> zero_grad."""
    from espnet2.schedulers.warmup_lr import WarmupLR

    cfg = CONFIGS[cfg_name]
    torch.manual_seed(0)
    model = build_reference_model(cfg)
    perturb_norms(model, torch.Generator().manual_seed(1000))
    sd0 = {k: v.clone() for k, v in model.state_dict().items()}
    opt = torch.optim.Adam(model.parameters(), lr=0.002, weight_decay=1e-6)
    sched = WarmupLR(opt, warmup_steps=10)
    model.train()
    rec = {"cfg": np.array(json.dumps(dict(cfg_name=cfg_name, lr=0.002, weight_decay=1e-6,
                                           warmup_steps=10, grad_clip=5.0, steps=steps)))}
    for k, v in sd0.items():
        rec["w." + k] = np32(v)
    for s in range(steps):
        batch = make_batch(cfg, torch.Generator().manual_seed(1 + s))
        for k, v in batch.items():
            rec[f"in{s}." + k] = v.clone().numpy()
        loss, stats, weight = model(**batch)
        loss.backward()
        gn = torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=5.0, norm_type=2.0)
        opt.step()
        sched.step()
        opt.zero_grad()
        rec[f"out{s}.loss"] = np32(loss)
        rec[f"out{s}.grad_norm"] = np32(gn)
        rec[f"out{s}.lr_after"] = np.array(opt.param_groups[0]["lr"], dtype=np.float64)
    for k, v in model.state_dict().items():
        rec["w_after." + k] = np32(v)
    path = os.path.join(OUT, f"{name}.npz")
    np.savez_compressed(path, **rec)
    print(f"{name}: -> {path} ({os.path.getsize(path)/1e6:.2f} MB)")


def capture_train_specaug(name="train3_specaug", cfg_name="tiny_hybrid", steps=3):
    """Three Trainer steps with SpecAug (conformer8 options) under one torch.manual_seed:
    the TimeWarp / mask draws of step k+1 come after step k's MultiSequential layer-drop
    draws (repeat.py:27: 2 encoder + 2 decoder uniforms per forward), so the parameters
    after step 3 pin the whole host RNG stream of the step, not only SpecAug's."""
    from espnet2.asr.specaug.specaug import SpecAug
    from espnet2.schedulers.warmup_lr import WarmupLR

    cfg = CONFIGS[cfg_name]
    torch.manual_seed(0)
    model = build_reference_model(cfg)
    perturb_norms(model, torch.Generator().manual_seed(1000))
    model.specaug = SpecAug(**SPECAUG_CONFS["conformer8"])
    sd0 = {k: v.clone() for k, v in model.state_dict().items()}
    opt = torch.optim.Adam(model.parameters(), lr=0.002, weight_decay=1e-6)
    sched = WarmupLR(opt, warmup_steps=10)
    model.train()
    rec = {"cfg": np.array(json.dumps(dict(cfg_name=cfg_name, lr=0.002, weight_decay=1e-6, warmup_steps=10,
                                           grad_clip=5.0, steps=steps, seed=123,
                                           specaug=SPECAUG_CONFS["conformer8"])))}
    for k, v in sd0.items():
        rec["w." + k] = np32(v)
    batches = [make_batch(cfg, torch.Generator().manual_seed(21 + s)) for s in range(steps)]
    torch.manual_seed(123)
    for s, batch in enumerate(batches):
        for k, v in batch.items():
            rec[f"in{s}." + k] = v.clone().numpy()
        loss, stats, weight = model(**{k: v.clone() for k, v in batch.items()})
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=5.0, norm_type=2.0)
        opt.step()
        sched.step()
        opt.zero_grad()
        rec[f"out{s}.loss"] = np32(loss)
    for k, v in model.state_dict().items():
        rec["w_after." + k] = np32(v)
    path = os.path.join(OUT, f"{name}.npz")
    np.savez_compressed(path, **rec)
    print(f"{name}: losses {[float(rec[f'out{s}.loss']) for s in range(steps)]} -> {path}")


def capture_ctc_op(name="ctc_op"):
    """Raw CTC (espnet2/asr/ctc.py:52-63 builtin path) on random logits, incl. repeated
    labels, a zero-length target and an infeasible target (zero_infinity=True -> 0)."""
    g = torch.Generator().manual_seed(7)
    T, B, V = 30, 5, 12
    logits = torch.randn(T, B, V, generator=g) * 2.0
    logits.requires_grad_(True)
    ilens = torch.tensor([30, 25, 30, 8, 17])
    olens = torch.tensor([6, 4, 0, 6, 9])  # utt3: 6 labels w/ repeats need >8 frames -> inf
    ys = [
        torch.tensor([3, 3, 5, 7, 7, 7]),
        torch.tensor([1, 2, 3, 4]),
        torch.tensor([], dtype=torch.long),
        torch.tensor([2, 2, 2, 2, 2, 2]),
        torch.tensor([4, 9, 4, 9, 4, 9, 11, 10, 1]),
    ]
    target = torch.cat(ys)
    lp = logits.log_softmax(2)
    ctc = torch.nn.CTCLoss(reduction="none", zero_infinity=True)
    loss_utt = ctc(lp, target, ilens, olens)
    loss = loss_utt.sum() / B
    loss.backward()
    rec = dict(logits=np32(logits), ilens=ilens.numpy(), olens=olens.numpy(),
               target=target.numpy(), loss_utt=np32(loss_utt), loss=np32(loss),
               grad_logits=np32(logits.grad))
    path = os.path.join(OUT, f"{name}.npz")
    np.savez_compressed(path, **rec)
    print(f"{name}: loss_utt={loss_utt.tolist()} -> {path}")


def capture_lsm_op(name="lsm_op"):
    """LabelSmoothingLoss (transformer/label_smoothing_loss.py:41-63) + th_accuracy
    (nets_utils.py:304-324) on random logits with ignore_id=-1 rows."""
    from espnet.nets.pytorch_backend.nets_utils import th_accuracy
    from espnet.nets.pytorch_backend.transformer.label_smoothing_loss import LabelSmoothingLoss

    g = torch.Generator().manual_seed(11)
    B, L, V = 3, 7, 23
    x = torch.randn(B, L, V, generator=g) * 3.0
    x.requires_grad_(True)
    tgt = torch.randint(0, V, (B, L), generator=g)
    tgt[0, 5:] = -1
    tgt[2, 2:] = -1
    rec = {}
    for sm, norm in ((0.1, False), (0.0, False), (0.2, True)):
        crit = LabelSmoothingLoss(V, -1, sm, normalize_length=norm)
        if x.grad is not None:
            x.grad = None
        loss = crit(x, tgt)
        loss.backward()
        tag = f"s{sm}_n{int(norm)}"
        rec[f"loss.{tag}"] = np32(loss)
        rec[f"grad.{tag}"] = np32(x.grad)
    rec["acc"] = np.array(th_accuracy(x.detach().view(-1, V), tgt, ignore_label=-1))
    rec["x"] = np32(x)
    rec["tgt"] = tgt.numpy()
    path = os.path.join(OUT, f"{name}.npz")
    np.savez_compressed(path, **rec)
    print(f"{name}: -> {path}")


def _ddp_worker(rank, world, init_file, cfg_name, out_path):
    import torch.distributed as dist
    from espnet2.torch_utils.recursive_op import recursive_average

    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank, world_size=world)
    cfg = CONFIGS[cfg_name]
    torch.manual_seed(0)
    model = build_reference_model(cfg)
    perturb_norms(model, torch.Generator().manual_seed(1000))
    ddp = torch.nn.parallel.DistributedDataParallel(model)
    ddp.train()
    full = make_batch(cfg, torch.Generator().manual_seed(1))
    # abs_task.py:1566-1575: each rank takes batch[rank::world_size] of the global batch
    batch = {k: v[rank::world] for k, v in full.items()}
    # collate crops padding to the local max (collate_fn.py pads per minibatch)
    tl = int(batch["speech_lengths"].max())
    batch["speech"] = batch["speech"][:, :tl].contiguous()
    loss, stats, weight = ddp(**batch)
    stats = {k: v for k, v in stats.items() if v is not None}
    # trainer.py:604-619
    loss = (loss * weight.type(loss.dtype)).sum()
    stats, weight = recursive_average(stats, weight, True)
    loss /= weight
    loss *= dist.get_world_size()
    loss.backward()
    if rank == 0:
        rec = {"cfg": np.array(json.dumps(dict(cfg_name=cfg_name, world=world)))}
        for k, v in full.items():
            rec["in." + k] = v.numpy()
        rec["out.loss_scaled"] = np32(loss)
        rec["out.weight"] = weight.numpy()
        for k, v in stats.items():
            rec["stat." + k] = np32(v)
        for k, p in model.named_parameters():
            rec["g." + k] = np32(p.grad)
        for k, v in model.state_dict().items():
            if "running" in k or "num_batches" in k:
                rec["buf_after." + k] = np32(v)
        np.savez_compressed(out_path, **rec)
    dist.destroy_process_group()


def capture_ddp(name="ddp2", cfg_name="tiny_hybrid"):
    import tempfile

    import torch.multiprocessing as mp

    init_file = tempfile.mktemp(prefix="ddp_init_")
    out_path = os.path.join(OUT, f"{name}.npz")
    mp.spawn(_ddp_worker, args=(2, init_file, cfg_name, out_path), nprocs=2, join=True)
    print(f"{name}: -> {out_path}")


SPECAUG_CONFS = {
    # egs2/librispeech/asr1/conf/tuning/train_asr_conformer8.yaml:62-76
    "conformer8": dict(apply_time_warp=True, time_warp_window=5, time_warp_mode="bicubic",
                       apply_freq_mask=True, freq_mask_width_range=[0, 27], num_freq_mask=2,
                       apply_time_mask=True, time_mask_width_ratio_range=[0.0, 0.05], num_time_mask=10),
    # fixed-width time masks (MaskAlongAxis on time), no warp
    "fixed_time": dict(apply_time_warp=False, apply_freq_mask=True, freq_mask_width_range=[0, 30],
                       num_freq_mask=2, apply_time_mask=True, time_mask_width_range=[0, 40], num_time_mask=2),
}


def capture_specaug(name="specaug"):
    """espnet2/asr/specaug/specaug.py under fixed torch seeds: equal-length batches (one
    warp for the batch), ragged batches (per-utterance warp + zero padding, including an
    utterance too short to warp) and the fixed-width time-mask variant."""
    from espnet2.asr.specaug.specaug import SpecAug

    cases = {
        "eq": ("conformer8", [120, 120, 120], 80, 11),
        "ragged": ("conformer8", [150, 97, 64, 9, 150], 80, 12),
        "eq_long": ("conformer8", [1000, 1000], 80, 13),
        "fixed": ("fixed_time", [200, 180], 80, 14),
    }
    out = {"cfg": np.array(json.dumps({"confs": SPECAUG_CONFS, "cases": cases}))}
    for key, (conf_name, lens, Fd, seed) in cases.items():
        gen = torch.Generator().manual_seed(100 + seed)
        T = max(lens)
        x = torch.randn(len(lens), T, Fd, generator=gen)
        for i, le in enumerate(lens):
            x[i, le:] = 0.0  # CommonCollateFn float_pad = 0.0
        xl = torch.tensor(lens, dtype=torch.long)
        torch.manual_seed(seed)
        y, yl = SpecAug(**SPECAUG_CONFS[conf_name])(x.clone(), xl)
        out[f"{key}.x"] = np32(x)
        out[f"{key}.lens"] = xl.numpy()
        out[f"{key}.y"] = np32(y)
    path = os.path.join(OUT, f"{name}.npz")
    np.savez_compressed(path, **out)
    print(f"{name}: {sorted(out)} -> {path}")


def capture_sampler(name="sampler"):
    """espnet2/samplers/num_elements_batch_sampler.py on synthetic shape files: speech
    (T, 80) and text (L,) shapes with ties, every sort option, min_batch_size
    redistribution, drop_last and padding=False."""
    import tempfile

    from espnet2.samplers.num_elements_batch_sampler import NumElementsBatchSampler

    rng = np.random.RandomState(5)
    n = 60
    Ts = rng.randint(200, 2001, size=n)
    Ts[5] = Ts[6] = Ts[7]  # ties keep file order
    d = tempfile.mkdtemp(prefix="shapes_")
    sp, tx = os.path.join(d, "speech_shape"), os.path.join(d, "text_shape")
    with open(sp, "w") as f:
        for i, t in enumerate(Ts):
            f.write(f"utt{i:03d} {t},80\n")
    with open(tx, "w") as f:
        for i, t in enumerate(Ts):
            f.write(f"utt{i:03d} {max(1, round(t / 25))}\n")
    settings = {
        "default": dict(batch_bins=400000, shape_files=[sp]),
        "two_files": dict(batch_bins=600000, shape_files=[sp, tx]),
        "desc_asc": dict(batch_bins=300000, shape_files=[sp], sort_in_batch="ascending", sort_batch="descending"),
        "min_bs": dict(batch_bins=1000000, shape_files=[sp], min_batch_size=9),
        "drop_last": dict(batch_bins=700000, shape_files=[sp], drop_last=True),
        "nopad": dict(batch_bins=500000, shape_files=[sp, tx], padding=False),
    }
    out = {"cfg": np.array(json.dumps({k: {kk: (vv if kk != "shape_files" else len(vv)) for kk, vv in v.items()}
                                       for k, v in settings.items()})),
           "T": Ts.astype(np.int64)}
    from espnet2.samplers.build_batch_sampler import build_batch_sampler
    # the other batch types, through build_batch_sampler (build_batch_sampler.py:72-162)
    cat = os.path.join(d, "utt2category")
    with open(cat, "w") as f:
        for i in range(n):
            f.write(f"utt{i:03d} {'a' if i % 3 else 'b'}\n")
    built = {
        "b_unsorted": dict(type="unsorted", batch_size=7, batch_bins=0, shape_files=[sp]),
        "b_unsorted_dl": dict(type="unsorted", batch_size=7, batch_bins=0, shape_files=[sp], drop_last=True),
        "b_sorted": dict(type="sorted", batch_size=7, batch_bins=0, shape_files=[sp]),
        "b_sorted_desc": dict(type="sorted", batch_size=8, batch_bins=0, shape_files=[sp], sort_batch="descending"),
        "b_folded": dict(type="folded", batch_size=12, batch_bins=0, shape_files=[sp, tx], fold_lengths=[800, 150]),
        "b_folded_min": dict(type="folded", batch_size=12, batch_bins=0, shape_files=[sp], fold_lengths=[500],
                             min_batch_size=3, sort_batch="descending", sort_in_batch="ascending"),
        "b_folded_cat": dict(type="folded", batch_size=10, batch_bins=0, shape_files=[sp], fold_lengths=[700],
                             utt2category_file=cat),
        "b_length": dict(type="length", batch_size=0, batch_bins=9000, shape_files=[sp, tx]),
        "b_length_min": dict(type="length", batch_size=0, batch_bins=20000, shape_files=[sp], min_batch_size=4),
        "b_length_nopad": dict(type="length", batch_size=0, batch_bins=7000, shape_files=[sp], padding=False,
                               drop_last=True),
        "b_numel": dict(type="numel", batch_size=0, batch_bins=600000, shape_files=[sp, tx], sort_batch="descending"),
    }
    for key, kw in built.items():
        s = build_batch_sampler(**kw)
        flat, sizes = [], []
        for b in s:
            flat += [int(k[3:]) for k in b]
            sizes.append(len(b))
        out[f"{key}.flat"] = np.array(flat, np.int64)
        out[f"{key}.sizes"] = np.array(sizes, np.int64)
    meta = json.loads(str(out["cfg"]))
    meta["built"] = {k: {kk: (vv if kk not in ("shape_files", "utt2category_file") else
                              (len(vv) if kk == "shape_files" else "utt2category"))
                         for kk, vv in v.items()} for k, v in built.items()}
    out["cfg"] = np.array(json.dumps(meta))
    for key, kw in settings.items():
        s = NumElementsBatchSampler(**kw)
        flat, sizes = [], []
        for b in s:
            flat += [int(k[3:]) for k in b]
            sizes.append(len(b))
        out[f"{key}.flat"] = np.array(flat, np.int64)
        out[f"{key}.sizes"] = np.array(sizes, np.int64)
    path = os.path.join(OUT, f"{name}.npz")
    np.savez_compressed(path, **out)
    print(f"{name}: {len(settings)} settings -> {path}")


def capture_frontend(name="frontend"):
    """espnet2/asr/frontend/default.py (Stft via torch.stft + LogMel with the restated
    librosa mel matrix, oracle/shim/librosa/filters.py) and espnet2/layers/global_mvn.py on
    ragged 16 kHz batches; two STFT settings (the 512/128 default and 400/160 windows)."""
    import tempfile

    from espnet2.asr.frontend.default import DefaultFrontend
    from espnet2.layers.global_mvn import GlobalMVN

    g = torch.Generator().manual_seed(21)
    out = {}
    cases = {"default": dict(fs=16000, n_fft=512, hop_length=128, n_mels=80),
             "win400": dict(fs=16000, n_fft=512, win_length=400, hop_length=160, n_mels=80, fmin=20, fmax=7600)}
    lens = [16000, 12345, 8000, 4097]
    x = torch.randn(len(lens), max(lens), generator=g) * 0.1
    for i, le in enumerate(lens):
        x[i, le:] = 0.0
    out["x"] = np32(x)
    out["lens"] = np.array(lens, np.int64)
    for key, conf in cases.items():
        fe = DefaultFrontend(**conf, frontend_conf=None)
        feats, flens = fe(x.clone(), torch.tensor(lens))
        out[f"{key}.feats"] = np32(feats)
        out[f"{key}.flens"] = flens.numpy()
        out[f"{key}.melmat"] = np32(fe.logmel.melmat)
    # GlobalMVN with an npz stats file of the default features
    f = out["default.feats"]
    fl = out["default.flens"]
    valid = np.concatenate([f[i, :fl[i]] for i in range(len(lens))], 0).astype(np.float64)
    d = tempfile.mkdtemp(prefix="mvn_")
    sp = os.path.join(d, "feats_stats.npz")
    np.savez(sp, count=np.array(valid.shape[0]), sum=valid.sum(0), sum_square=(valid ** 2).sum(0))
    mvn = GlobalMVN(sp)
    y, _ = mvn(torch.from_numpy(f).clone(), torch.from_numpy(fl))
    out["mvn.count"] = np.array(valid.shape[0])
    out["mvn.sum"] = valid.sum(0)
    out["mvn.sum_square"] = (valid ** 2).sum(0)
    out["mvn.y"] = np32(y)
    out["mvn.mean"] = mvn.mean.numpy()
    out["mvn.std"] = mvn.std.numpy()
    out["cfg"] = np.array(json.dumps({"cases": cases, "lens": lens}))
    path = os.path.join(OUT, f"{name}.npz")
    np.savez_compressed(path, **out)
    print(f"{name}: {sorted(out)} -> {path}")


def capture_avg_nbest(name="avg_nbest"):
    """espnet2/main_funcs/average_nbest_models.py on 4 epoch files of a small state dict
    (float weights + an int64 BatchNorm counter), criteria valid.loss min / valid.acc max,
    nbest [1, 2, 3] (the reference reuses the first loaded dict as accumulator)."""
    import tempfile
    from pathlib import Path

    from espnet2.main_funcs.average_nbest_models import average_nbest_models
    from espnet2.train.reporter import Reporter

    d = Path(tempfile.mkdtemp(prefix="avg_"))
    g = torch.Generator().manual_seed(9)
    rep = Reporter()
    losses = {1: 3.0, 2: 1.5, 3: 2.5, 4: 1.0}
    accs = {1: 0.5, 2: 0.7, 3: 0.9, 4: 0.6}
    out = {}
    for e in (1, 2, 3, 4):
        sd = {"w": torch.randn(5, 3, generator=g), "b": torch.randn(3, generator=g),
              "bn.num_batches_tracked": torch.tensor(10 * e, dtype=torch.long)}
        torch.save(sd, d / f"{e}epoch.pth")
        for k, v in sd.items():
            out[f"epoch{e}.{k}"] = v.numpy()
        rep.set_epoch(e)
        with rep.observe("valid") as sub:
            sub.register({"loss": losses[e], "acc": accs[e]})
    average_nbest_models(d, rep, [("valid", "loss", "min"), ("valid", "acc", "max")], [1, 2, 3])
    files = sorted(p.name for p in d.iterdir())
    links = {p.name: os.readlink(p) for p in d.iterdir() if p.is_symlink()}
    for f in files:
        if "ave" in f and not (d / f).is_symlink():
            sd = torch.load(d / f, map_location="cpu", weights_only=True)
            for k, v in sd.items():
                out[f"{f}.{k}"] = v.numpy()
    out["cfg"] = np.array(json.dumps({"losses": losses, "accs": accs, "files": files, "links": links}))
    path = os.path.join(OUT, f"{name}.npz")
    np.savez_compressed(path, **out)
    print(f"{name}: {files} -> {path}")


# --------------------------------------------------------------------------------------
# BASELINE-sized goldens (weights regenerated from the seed, not stored)
# --------------------------------------------------------------------------------------
SIZED = {
    # BASELINE.json configs[2] (C3): Conformer-L 12x512 + 6-layer decoder, V=5000, T=1000,
    # L=40, at B=2 with one ragged utterance (multi-tile T'=249, 12-layer depth)
    "c3_b2": dict(
        encoder="conformer", input_size=80, vocab_size=5000,
        encoder_conf=conformer_conf(512, 8, 2048, 12), decoder="transformer",
        decoder_conf=decoder_conf(8, 2048, 6),
        model_conf=dict(ctc_weight=0.3, lsm_weight=0.1, length_normalized_loss=False),
        speech_lengths=[1000, 871], text_lengths=[40, 33], seed=0,
    ),
    # BASELINE.json configs[1] (C2): Conformer-S 6x256, CTC only, T=500, L=20, at B=2
    "c2_b2": dict(
        encoder="conformer", input_size=80, vocab_size=5000,
        encoder_conf=conformer_conf(256, 4, 1024, 6), decoder="transformer",
        decoder_conf=decoder_conf(4, 2048, 6),
        model_conf=dict(ctc_weight=1.0, lsm_weight=0.0, length_normalized_loss=False),
        speech_lengths=[500, 437], text_lengths=[20, 14], seed=0,
    ),
    # BASELINE.json configs[4] (C5): Conformer-L + 6-layer decoder with SpecAug (conformer8),
    # a bucketed pair at the longest length of T ~ U[200, 2000] (T' = 499) and a ragged one,
    # L = round(T/25); the TimeWarp / mask draws and MultiSequential's layer-drop draws come
    # from torch.manual_seed(spec_seed) set before each forward
    "c5_b2": dict(
        encoder="conformer", input_size=80, vocab_size=5000,
        encoder_conf=conformer_conf(512, 8, 2048, 12), decoder="transformer",
        decoder_conf=decoder_conf(8, 2048, 6),
        model_conf=dict(ctc_weight=0.3, lsm_weight=0.1, length_normalized_loss=False),
        speech_lengths=[2000, 1317], text_lengths=[80, 53], seed=0,
        specaug="conformer8", spec_seed=77,
    ),
    # AMP check: d_k = 64, 2+2 blocks, T' = 99 (two 64-query tiles), ragged
    "amp_hybrid": dict(
        encoder="conformer", input_size=80, vocab_size=300,
        encoder_conf=conformer_conf(256, 4, 1024, 2), decoder="transformer",
        decoder_conf=decoder_conf(4, 1024, 2),
        model_conf=dict(ctc_weight=0.3, lsm_weight=0.1, length_normalized_loss=False),
        speech_lengths=[400, 360, 287], text_lengths=[20, 17, 9], seed=0,
    ),
}


def _rel_l2(a, b):
    a, b = a.double(), b.double()
    den = float(b.norm())
    return float((a - b).norm()) / den if den > 0 else float((a - b).norm())


def capture_sized(name):
    """A BASELINE-sized model in fp32 AND under torch.autocast("cpu", bfloat16).
    Weights come from torch.manual_seed(seed) + perturb_norms(Generator(1000 + seed)) —
    the build's modules initialise bit-identically under the same seed
    (tests/test_model_build.py) — and only per-tensor sums are stored to check the
    regeneration.  fp32: loss/stats/encoder output/CTC argmax, per-parameter gradient norm,
    sum and 256-element head, BN running stats.  bf16: loss/stats and, per parameter, the
    relative L2 distance of the autocast gradient from the fp32 one (the reference's own
    bf16 rounding error, the yardstick for the build's AMP path)."""
    cfg = SIZED[name]
    seed = cfg["seed"]
    torch.manual_seed(seed)
    model = build_reference_model(cfg)
    perturb_norms(model, torch.Generator().manual_seed(1000 + seed))
    if cfg.get("specaug"):
        from espnet2.asr.specaug.specaug import SpecAug
        model.specaug = SpecAug(**SPECAUG_CONFS[cfg["specaug"]])
        cfg = dict(cfg, specaug_conf=SPECAUG_CONFS[cfg["specaug"]])

    def reseed():  # the host draws of the step (SpecAug, then repeat.py:27), same for both passes
        if cfg.get("spec_seed") is not None:
            torch.manual_seed(cfg["spec_seed"])

    batch = make_batch(cfg, torch.Generator().manual_seed(1))
    model.train()
    sd0 = {k: v.clone() for k, v in model.state_dict().items()}
    rec = {"cfg": np.array(json.dumps({k: v for k, v in cfg.items()}))}
    for k, v in sd0.items():
        rec["wsum." + k] = np.array(v.double().sum().item())
    for k, v in batch.items():
        rec["in." + k] = v.numpy()
    enc_out = {}

    def enc_hook(mod, inp, out):
        enc_out["x"], enc_out["lens"] = out[0], out[1]

    h = model.encoder.register_forward_hook(enc_hook)
    reseed()
    loss, stats, weight = model(**{k: v.clone() for k, v in batch.items()})
    loss.backward()
    h.remove()
    rec["out.loss"] = np32(loss)
    rec["out.weight"] = weight.numpy()
    for k, v in stats.items():
        if v is not None:
            rec["stat." + k] = np32(v)
    rec["out.encoder_out"] = np32(enc_out["x"])
    rec["out.encoder_out_lens"] = enc_out["lens"].numpy()
    with torch.no_grad():
        logits = model.ctc.ctc_lo(enc_out["x"])
        rec["out.ctc_argmax"] = logits.argmax(-1).numpy()
        top2 = logits.topk(2, dim=-1).values
        rec["out.ctc_top2_gap"] = np32(top2[..., 0] - top2[..., 1])
    g32 = {}
    for k, p in model.named_parameters():
        if p.grad is None:
            continue
        g = p.grad.detach().clone()
        g32[k] = g
        rec["gn." + k] = np.array(g.double().norm().item())
        rec["gs." + k] = np.array(g.double().sum().item())
        rec["gh." + k] = np32(g.reshape(-1)[:256])
    for k, v in model.state_dict().items():
        if "running" in k or "num_batches" in k:
            rec["buf_after." + k] = np32(v)
    # the same step under CPU autocast (bf16), from the same initial state
    model.load_state_dict(sd0)
    model.zero_grad()
    reseed()
    with torch.autocast("cpu", dtype=torch.bfloat16):
        aloss, astats, _ = model(**{k: v.clone() for k, v in batch.items()})
    aloss.backward()
    rec["amp.loss"] = np32(aloss)
    for k, v in astats.items():
        if v is not None:
            rec["ampstat." + k] = np32(v)
    for k, p in model.named_parameters():
        if k in g32:
            rec["ampdev." + k] = np.array(_rel_l2(p.grad.detach(), g32[k]))
    path = os.path.join(OUT, f"{name}.npz")
    np.savez_compressed(path, **rec)
    devs = sorted(float(rec[k]) for k in rec if k.startswith("ampdev."))
    print(f"{name}: loss={loss.item():.6f} amp={aloss.item():.6f} ampdev median {devs[len(devs) // 2]:.2e} "
          f"max {devs[-1]:.2e} -> {path} ({os.path.getsize(path) / 1e6:.2f} MB)")


def capture_epoch(name="epoch_accum2", cfg_name="tiny_hybrid"):
    """Trainer.train_one_epoch (espnet2/train/trainer.py:472-731) itself, on the CPU, over a
    fixed 4-batch iterator with accum_grad=2 (the conformer8 recipe uses 4): loss / accum,
    two backwards per update, clip_grad_norm_(5), Adam + WarmupLR after every 2nd batch;
    then the reporter's per-epoch aggregates (reporter.py) and the parameters after."""
    import argparse

    from espnet2.schedulers.warmup_lr import WarmupLR
    from espnet2.train.reporter import Reporter
    from espnet2.train.trainer import Trainer, TrainerOptions
    from espnet2.train.distributed_utils import DistributedOption

    cfg = CONFIGS[cfg_name]
    torch.manual_seed(0)
    model = build_reference_model(cfg)
    perturb_norms(model, torch.Generator().manual_seed(1000))
    sd0 = {k: v.clone() for k, v in model.state_dict().items()}
    opt = torch.optim.Adam(model.parameters(), lr=0.002, weight_decay=1e-6)
    sched = WarmupLR(opt, warmup_steps=10)
    batches = [make_batch(cfg, torch.Generator().manual_seed(11 + s)) for s in range(4)]
    rec = {"cfg": np.array(json.dumps(dict(cfg_name=cfg_name, lr=0.002, weight_decay=1e-6, warmup_steps=10,
                                           grad_clip=5.0, accum_grad=2, n_batches=4)))}
    for k, v in sd0.items():
        rec["w." + k] = np32(v)
    for s, b in enumerate(batches):
        for k, v in b.items():
            rec[f"in{s}." + k] = v.clone().numpy()
    args = argparse.Namespace(ngpu=0, resume=False, use_amp=False, train_dtype="float32", grad_noise=False,
                              accum_grad=2, grad_clip=5.0, grad_clip_type=2.0, log_interval=None,
                              no_forward_run=False, use_matplotlib=False, use_tensorboard=False, use_wandb=False,
                              output_dir="/tmp", max_epoch=1, seed=0, sharded_ddp=False, patience=None,
                              keep_nbest_models=[1], nbest_averaging_interval=0,
                              early_stopping_criterion=("valid", "loss", "min"),
                              best_model_criterion=[("train", "loss", "min")],
                              val_scheduler_criterion=("valid", "loss"), unused_parameters=False,
                              wandb_model_log_interval=-1, create_graph_in_tensorboard=False)
    options = TrainerOptions(**{f: getattr(args, f) for f in TrainerOptions.__dataclass_fields__})
    reporter = Reporter()
    reporter.set_epoch(1)
    iterator = [([f"u{s}_{i}" for i in range(len(b["speech"]))], {k: v.clone() for k, v in b.items()})
                for s, b in enumerate(batches)]
    with reporter.observe("train") as sub:
        invalid = Trainer.train_one_epoch(model=model, iterator=iterator, optimizers=[opt], schedulers=[sched],
                                          scaler=None, reporter=sub, summary_writer=None, options=options,
                                          distributed_option=DistributedOption(distributed=False))
    stats = reporter.stats[1]["train"]
    keys = [k for k, v in stats.items() if isinstance(v, float) and not k.endswith("_time")]
    rec["stats_keys"] = np.array(json.dumps(keys))
    for k in keys:
        rec["stat." + k] = np.array(stats[k], dtype=np.float64)
    rec["all_invalid"] = np.array(bool(invalid))
    rec["total_count"] = np.array(stats["total_count"])
    rec["time_keys"] = np.array(json.dumps(sorted(k for k in stats if k.endswith("_time"))))
    for k, v in model.state_dict().items():
        rec["w_after." + k] = np32(v)
    path = os.path.join(OUT, f"{name}.npz")
    np.savez_compressed(path, **rec)
    print(f"{name}: stats {({k: stats[k] for k in keys})} -> {path}")


def capture_reporter(name="reporter"):
    """espnet2/train/reporter.py: SubReporter aggregation (WeightedAverage with NaN / inf
    values and zero weights, Average, keys registered late or skipped in a step), its
    log_message, and Reporter epoch bookkeeping (sort / best / early stopping)."""
    from espnet2.train.reporter import Reporter
    rep = Reporter()
    seq = [  # (weighted stats, weight, unweighted stats)
        ({"loss": 3.0, "acc": 0.5}, 4, {"lr": 0.1}),
        ({"loss": float("nan"), "acc": 0.25}, 2, {"lr": 0.2}),
        ({"loss": 1.0, "acc": None}, 3, {}),
        ({"loss": 2.0, "acc": 0.75, "late": 9.0}, 1, {"lr": 0.4}),
        ({"loss": float("inf"), "acc": 1.0, "late": 1.0}, 5, {"lr": 0.5}),
    ]
    out = {}
    msgs = []
    for e in (1, 2, 3):
        rep.set_epoch(e)
        with rep.observe("train") as sub:
            for st, w, un in seq:
                sub.register({k: (None if v is None else v * e) for k, v in st.items()}, w)
                if un:
                    sub.register(un)
                sub.next()
                msgs.append(sub.log_message(-2))
        with rep.observe("valid") as sub:
            sub.register({"loss": float(4 - e) if e != 2 else 5.0, "acc": 0.1 * e}, 2)
            sub.next()
    for e in (1, 2, 3):
        for key in ("train", "valid"):
            for k2, v in rep.stats[e][key].items():
                if isinstance(v, float):
                    out[f"e{e}.{key}.{k2}"] = np.array(v, dtype=np.float64)
    out["msgs"] = np.array(json.dumps(msgs))
    out["sort_valid_loss_min"] = np.array(rep.sort_epochs("valid", "loss", "min"))
    out["best_train_acc_max"] = np.array(rep.get_best_epoch("train", "acc", "max"))
    out["early_stop_p0"] = np.array(rep.check_early_stopping(0, "valid", "loss", "min"))
    out["early_stop_p1"] = np.array(rep.check_early_stopping(1, "valid", "loss", "min"))
    path = os.path.join(OUT, f"{name}.npz")
    np.savez_compressed(path, **out)
    print(f"{name}: {len(out)} entries -> {path}")


def capture_iter_factory(name="iterfactory"):
    """SequenceIterFactory batch orders (espnet2/iterators/sequence_iter_factory.py:72-135)
    for shuffle on/off and num_iters_per_epoch below / above the number of batches."""
    from espnet2.iterators.sequence_iter_factory import SequenceIterFactory
    batches = [tuple(f"u{i}_{j}" for j in range(i % 3 + 1)) for i in range(7)]
    out = {}
    cases = {"plain": dict(), "shuffle": dict(shuffle=True), "n3": dict(shuffle=True, num_iters_per_epoch=3),
             "n10": dict(shuffle=True, num_iters_per_epoch=10), "n3_noshuf": dict(num_iters_per_epoch=3)}
    for key, kw in cases.items():
        f = SequenceIterFactory(dataset=None, batches=list(batches), seed=5, **kw)
        for epoch in range(1, 6):
            import espnet2.iterators.sequence_iter_factory as m
            orig = m.DataLoader
            got = {}
            m.DataLoader = lambda dataset, batch_sampler, **k: got.setdefault("b", batch_sampler)
            try:
                f.build_iter(epoch)
            finally:
                m.DataLoader = orig
            out[f"{key}.e{epoch}"] = np.array(json.dumps([list(b) for b in got["b"]]))
    out["cfg"] = np.array(json.dumps({"batches": [list(b) for b in batches], "cases": cases, "seed": 5}))
    path = os.path.join(OUT, f"{name}.npz")
    np.savez_compressed(path, **out)
    print(f"{name}: {len(out)} entries -> {path}")


# (beam, length_bonus weight, maxlenratio[, ctc_weight])
BEAM_CASES = [(3, 0.0, 0.0), (4, 0.5, 0.0), (3, 0.0, 0.5), (3, 0.0, 0.0, 0.3), (4, 0.5, 0.0, 0.5),
              (3, 0.0, 0.5, 0.3)]


def capture_beam(name="beam", cfg_name="tiny_hybrid"):
    """espnet/nets/beam_search.py BeamSearch on the tiny hybrid model (weights of the
    tiny_hybrid golden, eval mode), scorers: decoder (weight 1) + LengthBonus; each
    utterance encoded alone as Speech2Text does.  Records every n-best hypothesis."""
    from espnet.nets.beam_search import BeamSearch
    from espnet.nets.scorers.ctc import CTCPrefixScorer
    from espnet.nets.scorers.length_bonus import LengthBonus
    z = np.load(os.path.join(OUT, cfg_name + ".npz"))
    cfg = json.loads(str(z["cfg"]))
    model = build_reference_model(cfg)
    model.load_state_dict({k[2:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("w.")})
    model.eval()
    speech = torch.from_numpy(z["in.speech"])
    lens = torch.from_numpy(z["in.speech_lengths"])
    V = model.vocab_size
    out = {}
    meta = []
    with torch.no_grad():
        for ci, case in enumerate(BEAM_CASES):
            beam, lb, mlr = case[:3]
            cw = case[3] if len(case) > 3 else 0.0
            bs = BeamSearch(scorers={"decoder": model.decoder, "ctc": CTCPrefixScorer(model.ctc, model.eos),
                                     "length_bonus": LengthBonus(V)},
                            weights={"decoder": 1.0 - cw, "ctc": cw, "length_bonus": lb}, beam_size=beam,
                            vocab_size=V, sos=model.sos, eos=model.eos, token_list=None,
                            pre_beam_score_key="full")
            for u in range(speech.shape[0]):
                le = int(lens[u])
                enc, _ = model.encode(speech[u:u + 1, :le], lens[u:u + 1])
                nbest = bs(x=enc[0], maxlenratio=mlr, minlenratio=0.0)
                for r, h in enumerate(nbest):
                    key = f"c{ci}.u{u}.h{r}"
                    out[key + ".yseq"] = h.yseq.numpy().astype(np.int64)
                    out[key + ".score"] = np.float64(float(h.score))
                    out[key + ".decoder"] = np.float64(float(h.scores["decoder"]))
                    if cw:
                        out[key + ".ctc"] = np.float64(float(h.scores["ctc"]))
                meta.append({"case": ci, "utt": u, "n": len(nbest)})
    out["cfg"] = np.array(json.dumps({"cases": BEAM_CASES, "nbest": meta, "model": cfg_name}))
    path = os.path.join(OUT, f"{name}.npz")
    np.savez_compressed(path, **out)
    print(f"{name}: {len(meta)} searches -> {path}")


def capture_ctc_th(name="ctc_th"):
    """espnet/nets/ctc_prefix_score.py CTCPrefixScoreTH (the vectorised prefix scorer the
    reference's BatchBeamSearch uses through CTCPrefixScorer.batch_score_partial) on seeded
    log-posteriors of two utterances of different lengths: three steps (full vocabulary, a
    pre-beam subset, full again) with index_select_state between them, including a selected
    label outside the scored subset (its state falls back to candidate 0, as the reference
    does).  Records every step's local scores."""
    from espnet.nets.ctc_prefix_score import CTCPrefixScoreTH
    g = torch.Generator().manual_seed(5)
    B, T, O, W = 2, 23, 9, 3
    eos = O - 1
    x = torch.log_softmax(torch.randn(B, T, O, generator=g) * 2.0, dim=-1)
    xlens = torch.tensor([23, 17])
    out = {"x": np32(x), "xlens": xlens.numpy().astype(np.int64)}
    impl = CTCPrefixScoreTH(x.clone(), xlens, 0, eos)
    n_bh = B * W
    y = [torch.tensor([eos]) for _ in range(n_bh)]
    state = None
    plan = [None, torch.tensor([[1, 2, 3, 8], [2, 4, 5, 6], [1, 3, 5, 7], [2, 3, 4, 5], [1, 6, 7, 8],
                                [3, 4, 6, 7]]), None]
    best_plan = [torch.tensor([[1, 9 + 2, 18 + 3], [4, 9 + 5, 18 + 7]]),
                 torch.tensor([[2, 9 + 4, 18 + 6], [3 + 9, 18 + 7, 8]]),
                 None]
    for step, sids in enumerate(plan):
        sc, st = impl(y, state, sids)
        out[f"s{step}.scores"] = np32(sc)
        out[f"s{step}.y"] = np.stack([yy.numpy() for yy in y]).astype(np.int64)
        if sids is not None:
            out[f"s{step}.ids"] = sids.numpy().astype(np.int64)
        best = best_plan[step]
        if best is None:
            break
        out[f"s{step}.best"] = best.numpy().astype(np.int64)
        state = impl.index_select_state(st, best)
        hyp = (best // O + (torch.arange(B) * W).view(-1, 1)).view(-1)
        lab = torch.fmod(best, O).view(-1)
        y = [torch.cat([y[int(h)], lab[i:i + 1]]) for i, h in enumerate(hyp)]
    out["cfg"] = np.array(json.dumps({"B": B, "T": T, "O": O, "W": W, "eos": eos, "blank": 0}))
    path = os.path.join(OUT, f"{name}.npz")
    np.savez_compressed(path, **out)
    print(f"{name} -> {path}")


def capture_ctc_th_ext(name="ctc_th_ext"):
    """CTCPrefixScoreTH's attention-windowed scoring (margin > 0 with att_w,
    espnet/nets/ctc_prefix_score.py:57-62, 143-153) and its streaming extension (extend_prob /
    extend_state, :222-269, driven per hypothesis as scorers/ctc.py:128-158 does), on seeded
    log-posteriors.  Window case: two utterances (30 and 21 frames), margin 3, attention
    weights peaked on a centre that advances each step, three steps with index_select_state
    between them.  Streaming case: one utterance revealed 12 -> 20 -> 30 frames, one step per
    chunk, the selected hypotheses' states extended before each new chunk's step."""
    from espnet.nets.ctc_prefix_score import CTCPrefixScoreTH
    g = torch.Generator().manual_seed(11)
    out = {}
    # --- window
    B, T, O, W, margin = 2, 30, 9, 3, 3
    eos = O - 1
    x = torch.log_softmax(torch.randn(B, T, O, generator=g) * 2.0, dim=-1)
    xlens = torch.tensor([30, 21])
    out["w.x"] = np32(x)
    out["w.xlens"] = xlens.numpy().astype(np.int64)
    impl = CTCPrefixScoreTH(x.clone(), xlens, 0, eos, margin=margin)
    n_bh = B * W
    y = [torch.tensor([eos]) for _ in range(n_bh)]
    state = None
    plan = [None, torch.tensor([[1, 2, 3, 8], [2, 4, 5, 6], [1, 3, 5, 7], [2, 3, 4, 5], [1, 6, 7, 8],
                                [3, 4, 6, 7]]), None]
    best_plan = [torch.tensor([[1, 9 + 2, 18 + 3], [4, 9 + 5, 18 + 7]]),
                 torch.tensor([[2, 9 + 4, 18 + 6], [3 + 9, 18 + 7, 8]]), None]
    frames = torch.arange(T, dtype=torch.float32)
    for step, sids in enumerate(plan):
        centre = 4.0 + 6.0 * step + torch.rand(n_bh, 1, generator=g) * 3.0
        att_w = torch.softmax(-((frames.view(1, -1) - centre) ** 2) / 4.0, dim=-1)
        sc, st = impl(y, state, sids, att_w)
        out[f"w.s{step}.att_w"] = np32(att_w)
        out[f"w.s{step}.scores"] = np32(sc)
        out[f"w.s{step}.y"] = np.stack([yy.numpy() for yy in y]).astype(np.int64)
        out[f"w.s{step}.fminmax"] = np.array([st[2], st[3]], dtype=np.int64)
        if sids is not None:
            out[f"w.s{step}.ids"] = sids.numpy().astype(np.int64)
        best = best_plan[step]
        if best is None:
            break
        out[f"w.s{step}.best"] = best.numpy().astype(np.int64)
        state = impl.index_select_state(st, best)
        hyp = (best // O + (torch.arange(B) * W).view(-1, 1)).view(-1)
        lab = torch.fmod(best, O).view(-1)
        y = [torch.cat([y[int(h)], lab[i:i + 1]]) for i, h in enumerate(hyp)]
    # --- streaming
    T, W = 30, 3
    xs = torch.log_softmax(torch.randn(1, T, O, generator=g) * 2.0, dim=-1)
    out["s.x"] = np32(xs)
    chunks = [12, 20, 30]
    impl = CTCPrefixScoreTH(xs[:, :chunks[0]].clone(), torch.tensor([chunks[0]]), 0, eos)
    y = [torch.tensor([eos]) for _ in range(W)]
    state = None
    best_plan = [torch.tensor([[1, 9 + 2, 18 + 3]]), torch.tensor([[2, 9 + 4, 18 + 6]]), None]
    for step, tc in enumerate(chunks):
        if step > 0:
            impl.extend_prob(xs[:, :tc].clone())
            per = [impl.extend_state((state[0][:, :, i], state[1][i], state[2], state[3])) for i in range(W)]
            state = (torch.stack([s[0] for s in per], dim=2), torch.stack([s[1] for s in per]), per[0][2], per[0][3])
        sc, st = impl(y, state, None)
        out[f"s.s{step}.scores"] = np32(sc)
        out[f"s.s{step}.y"] = np.stack([yy.numpy() for yy in y]).astype(np.int64)
        best = best_plan[step]
        if best is None:
            break
        out[f"s.s{step}.best"] = best.numpy().astype(np.int64)
        state = impl.index_select_state(st, best)
        lab = torch.fmod(best, O).view(-1)
        hyp = (best // O).view(-1)
        y = [torch.cat([y[int(h)], lab[i:i + 1]]) for i, h in enumerate(hyp)]
    out["cfg"] = np.array(json.dumps({"B": B, "O": O, "W": W, "eos": eos, "blank": 0, "margin": margin,
                                      "chunks": chunks}))
    path = os.path.join(OUT, f"{name}.npz")
    np.savez_compressed(path, **out)
    print(f"{name} -> {path}")


def capture_beam_batch(name="beam_batch", cfg_name="tiny_hybrid"):
    """espnet/nets/batch_beam_search.py BatchBeamSearch (decoder batch_score, CTCPrefixScorer
    batch_score_partial over CTCPrefixScoreTH, LengthBonus) on the tiny hybrid model, the
    BEAM_CASES of capture_beam with CTC weight > 0."""
    from espnet.nets.batch_beam_search import BatchBeamSearch
    from espnet.nets.scorers.ctc import CTCPrefixScorer
    from espnet.nets.scorers.length_bonus import LengthBonus
    z = np.load(os.path.join(OUT, cfg_name + ".npz"))
    cfg = json.loads(str(z["cfg"]))
    model = build_reference_model(cfg)
    model.load_state_dict({k[2:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("w.")})
    model.eval()
    speech = torch.from_numpy(z["in.speech"])
    lens = torch.from_numpy(z["in.speech_lengths"])
    V = model.vocab_size
    cases = [c for c in BEAM_CASES if len(c) > 3] + [(3, 0.0, 0.0, 1.0)]
    out, meta = {}, []
    with torch.no_grad():
        for ci, case in enumerate(cases):
            beam, lb, mlr, cw = case
            bs = BatchBeamSearch(scorers={"decoder": model.decoder, "ctc": CTCPrefixScorer(model.ctc, model.eos),
                                          "length_bonus": LengthBonus(V)},
                                 weights={"decoder": 1.0 - cw, "ctc": cw, "length_bonus": lb}, beam_size=beam,
                                 vocab_size=V, sos=model.sos, eos=model.eos, token_list=None,
                                 pre_beam_score_key="full")
            for u in range(speech.shape[0]):
                le = int(lens[u])
                enc, _ = model.encode(speech[u:u + 1, :le], lens[u:u + 1])
                nbest = bs(x=enc[0], maxlenratio=mlr, minlenratio=0.0)
                for r, h in enumerate(nbest):
                    key = f"c{ci}.u{u}.h{r}"
                    out[key + ".yseq"] = h.yseq.numpy().astype(np.int64)
                    out[key + ".score"] = np.float64(float(h.score))
                meta.append({"case": ci, "utt": u, "n": len(nbest)})
    out["cfg"] = np.array(json.dumps({"cases": cases, "nbest": meta, "model": cfg_name}))
    path = os.path.join(OUT, f"{name}.npz")
    np.savez_compressed(path, **out)
    print(f"{name}: {len(meta)} searches -> {path}")


def capture_lm(name="lm_tiny", cfg_name="tiny_hybrid"):
    """espnet2/lm/transformer_lm.py TransformerLM (pos_enc None as in the librispeech lm_conf,
    2 layers, att_unit 128 / 2 heads so d_k = 64) over the tiny hybrid model's vocabulary:
    forward logits, batch_score on prefixes, and BeamSearch with LM shallow fusion
    (scorers decoder + ctc + lm + length_bonus, asr_inference.py:140-183)."""
    from espnet.nets.beam_search import BeamSearch
    from espnet.nets.scorers.ctc import CTCPrefixScorer
    from espnet.nets.scorers.length_bonus import LengthBonus
    from espnet2.lm.transformer_lm import TransformerLM
    z = np.load(os.path.join(OUT, cfg_name + ".npz"))
    cfg = json.loads(str(z["cfg"]))
    model = build_reference_model(cfg)
    model.load_state_dict({k[2:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("w.")})
    model.eval()
    V = model.vocab_size
    torch.manual_seed(3)
    lm_conf = dict(vocab_size=V, pos_enc=None, embed_unit=32, att_unit=128, head=2, unit=256, layer=2,
                   dropout_rate=0.0)
    lm = TransformerLM(**lm_conf)
    gen = torch.Generator().manual_seed(4)
    with torch.no_grad():
        for n, p_ in lm.named_parameters():  # non-trivial norms
            if "norm" in n or "embed.1" in n:
                p_.add_(torch.randn(p_.shape, generator=gen) * 0.1)
    lm.eval()
    out = {f"w.{k}": np32(v) for k, v in lm.state_dict().items()}
    ids = torch.randint(2, V - 1, (3, 7), generator=gen)
    ys = torch.cat([torch.full((4, 1), model.sos), torch.randint(2, V - 1, (4, 4), generator=gen)], dim=1)
    with torch.no_grad():
        logits, _ = lm(ids, None)
        logp, _ = lm.batch_score(ys, [None] * 4, None)
    out["in.ids"] = ids.numpy().astype(np.int64)
    out["in.ys"] = ys.numpy().astype(np.int64)
    out["out.logits"] = np32(logits)
    out["out.bs_logp"] = np32(logp)
    speech = torch.from_numpy(z["in.speech"])
    lens = torch.from_numpy(z["in.speech_lengths"])
    cases = [(3, 0.0, 0.0, 0.3, 0.3), (4, 0.5, 0.0, 0.5, 0.5)]
    meta = []
    with torch.no_grad():
        for ci, (beam, lb, mlr, cw, lw) in enumerate(cases):
            bs = BeamSearch(scorers={"decoder": model.decoder, "ctc": CTCPrefixScorer(model.ctc, model.eos),
                                     "lm": lm, "length_bonus": LengthBonus(V)},
                            weights={"decoder": 1.0 - cw, "ctc": cw, "lm": lw, "length_bonus": lb},
                            beam_size=beam, vocab_size=V, sos=model.sos, eos=model.eos, token_list=None,
                            pre_beam_score_key="full")
            for u in range(speech.shape[0]):
                le = int(lens[u])
                enc, _ = model.encode(speech[u:u + 1, :le], lens[u:u + 1])
                nbest = bs(x=enc[0], maxlenratio=mlr, minlenratio=0.0)
                for r, h in enumerate(nbest):
                    key = f"c{ci}.u{u}.h{r}"
                    out[key + ".yseq"] = h.yseq.numpy().astype(np.int64)
                    out[key + ".score"] = np.float64(float(h.score))
                    out[key + ".lm"] = np.float64(float(h.scores["lm"]))
                meta.append({"case": ci, "utt": u, "n": len(nbest)})
    out["cfg"] = np.array(json.dumps({"lm_conf": lm_conf, "cases": cases, "nbest": meta, "model": cfg_name}))
    path = os.path.join(OUT, f"{name}.npz")
    np.savez_compressed(path, **out)
    print(f"{name}: {len(meta)} searches -> {path}")


if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    which = sys.argv[1:] or ["models", "train", "ops", "ddp"]
    for n, c in CONFIGS.items():
        if "models" in which or n in which:
            capture_model(n, c, light=n.startswith("medium"))
    if "train" in which:
        capture_train_steps()
    if "ops" in which:
        capture_ctc_op()
        capture_lsm_op()
    if "ddp" in which:
        capture_ddp()
    if "specaug" in which:
        capture_specaug()
    if "sampler" in which:
        capture_sampler()
    if "avg" in which:
        capture_avg_nbest()
    if "frontend" in which:
        capture_frontend()
    if "beam" in which:
        capture_beam()
    if "ctc_th" in which:
        capture_ctc_th()
    if "ctc_th_ext" in which:
        capture_ctc_th_ext()
    if "beam_batch" in which:
        capture_beam_batch()
    if "lm" in which:
        capture_lm()
    if "train_specaug" in which:
        capture_train_specaug()
    if "epoch" in which:
        capture_epoch()
    if "reporter" in which:
        capture_reporter()
    if "iterfactory" in which:
        capture_iter_factory()
    for n in SIZED:
        if n in which or "sized" in which:
            capture_sized(n)
