"""Benchmark: ESPnet2 ASR training step (ESPnetASRModel, Conformer-L + Transformer decoder,
hybrid CTC/attention) on MI355X — BASELINE.json metric "utterances/sec + step-time,
Conformer-L T=1000 batch=32 @1/2/4/8 GPU".

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2] [--fp32]
    torchrun --nproc-per-node N bench.py --gpus N ...      (one rank per GPU, RCCL)

A step = forward + backward + RCCL gradient all-reduce (N>1) + clip_grad_norm(5) + Adam +
WarmupLR + zero_grad over one synthetic batch per rank (speech ~ N(0,1) (32, 1000, 80),
text uniform in [2, V-2], L=40 — SURVEY.md §8d), inputs resident in HBM before timing.
Weak scaling: 32 utterances per GPU.  Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "espnet-1_amd"))
sys.path.insert(0, ROOT)

import espnet_amd  # noqa: E402,F401  (process-group settings for the captured DP step, before any init)
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "utterances/sec + step-time, Conformer-L T=1000 batch=32 @1/2/4/8 GPU"
PEAK = {"bf16": 2500.0, "f32": 157.3}  # dense MFMA TFLOP/s, MI355X_MICROARCH.md


def c3_config():
    """egs2/librispeech/asr1/conf/tuning/train_asr_conformer8.yaml:2-34 with input_size 80."""
    return dict(
        input_size=80, vocab_size=5000, B=32, T=1000, L=40,
        encoder_conf=dict(output_size=512, attention_heads=8, linear_units=2048, num_blocks=12,
                          dropout_rate=0.1, positional_dropout_rate=0.1, attention_dropout_rate=0.1,
                          input_layer="conv2d", normalize_before=True, macaron_style=True,
                          rel_pos_type="latest", pos_enc_layer_type="rel_pos",
                          selfattention_layer_type="rel_selfattn", activation_type="swish",
                          use_cnn_module=True, cnn_module_kernel=31),
        decoder="transformer",
        decoder_conf=dict(attention_heads=8, linear_units=2048, num_blocks=6, dropout_rate=0.1,
                          positional_dropout_rate=0.1, self_attention_dropout_rate=0.1,
                          src_attention_dropout_rate=0.1),
        model_conf=dict(ctc_weight=0.3, lsm_weight=0.1, length_normalized_loss=False),
        optim=dict(lr=0.0025, weight_decay=1e-6), warmup_steps=40000,
        gflop_per_step=6643.0,
    )


def _diag_dropout(cfg):
    """EA_BENCH_DIAG_DROPOUT=x: every dropout rate set to x — a diagnostic A/B of what the
    dropout costs (the bench line then names the rate in `config`; never the reported run)."""
    x = os.environ.get("EA_BENCH_DIAG_DROPOUT")
    if x is None:
        return cfg
    for k in ("encoder_conf", "decoder_conf"):
        for kk in list(cfg[k]):
            if "dropout_rate" in kk:
                cfg[k][kk] = float(x)
    return cfg


def c2_config():
    c = c3_config()
    c.update(B=16, T=500, L=20, decoder=None, gflop_per_step=282.8)
    c["encoder_conf"] = dict(c["encoder_conf"], output_size=256, attention_heads=4, linear_units=1024,
                             num_blocks=6)
    c["model_conf"] = dict(ctc_weight=1.0, lsm_weight=0.0, length_normalized_loss=False)
    return c


def c5_config():
    """BASELINE.json configs[4] / SURVEY.md §8d C5: Conformer-L + SpecAug (conformer8.yaml:62-76),
    bucketed variable-length utterances T ~ U[200, 2000], L = round(T/25), NumElements
    batching with batch_bins sized so a batch holds ~32 utterances at T=1000 (per GPU)."""
    c = c3_config()
    c.update(B=None, T=2000, L=80, gflop_per_step=None, corpus=640, batch_bins=32 * 1000 * 80,
             specaug_conf=dict(apply_time_warp=True, time_warp_window=5, time_warp_mode="bicubic",
                               apply_freq_mask=True, freq_mask_width_range=[0, 27], num_freq_mask=2,
                               apply_time_mask=True, time_mask_width_ratio_range=[0.0, 0.05],
                               num_time_mask=10))
    return c


def c5_batches(cfg, rank, world, seed=7):
    """Synthetic LibriSpeech-shaped corpus -> NumElementsBatchSampler batches (host), this
    rank's share (batch[rank::world] of each global batch, abs_task.py:1566-1575)."""
    from espnet_amd.samplers.num_elements_batch_sampler import NumElementsBatchSampler
    g = torch.Generator().manual_seed(seed)
    n, V, F = cfg["corpus"], cfg["vocab_size"], cfg["input_size"]
    Ts = torch.randint(200, 2001, (n,), generator=g).tolist()
    shapes = {f"utt{i:04d}": [t, F] for i, t in enumerate(Ts)}
    sampler = NumElementsBatchSampler(cfg["batch_bins"] * world, utt2shapes=[shapes])
    order = torch.randperm(len(sampler), generator=g).tolist()  # SequenceIterFactory shuffles batches
    batches = []
    for bi in order:
        keys = list(sampler.batch_list[bi])[rank::world]
        if not keys:
            continue
        lens = [shapes[k][0] for k in keys]
        Ls = [max(1, round(t / 25)) for t in lens]
        B, T, L = len(keys), max(lens), max(Ls)
        speech = torch.zeros(B, T, F)
        text = torch.full((B, L), -1, dtype=torch.long)
        for i, (t, l) in enumerate(zip(lens, Ls)):
            speech[i, :t] = torch.randn(t, F, generator=g)
            text[i, :l] = torch.randint(2, V - 1, (l,), generator=g)
        batches.append(dict(speech=speech, speech_lengths=torch.tensor(lens), text=text,
                            text_lengths=torch.tensor(Ls), _lens_host=lens, _maxlens=(T, L)))
    return batches


def token_list(V):
    return ["<blank>", "<unk>"] + [f"t{i}" for i in range(V - 3)] + ["<sos/eos>"]


def build(cfg, seed=0):
    from espnet_amd.tasks.asr import build_model
    torch.manual_seed(seed)
    args = dict(token_list=token_list(cfg["vocab_size"]), input_size=cfg["input_size"], encoder="conformer",
                encoder_conf=cfg["encoder_conf"], decoder=cfg["decoder"],
                decoder_conf=cfg["decoder_conf"], model_conf=cfg["model_conf"], normalize="utterance_mvn",
                specaug="specaug" if cfg.get("specaug_conf") else None, specaug_conf=cfg.get("specaug_conf"))
    return build_model(args)


def synthetic_batch(cfg, seed):
    g = torch.Generator().manual_seed(seed)
    B, T, L, V = cfg["B"], cfg["T"], cfg["L"], cfg["vocab_size"]
    return dict(speech=torch.randn(B, T, cfg["input_size"], generator=g),
                speech_lengths=torch.full((B,), T, dtype=torch.long),
                text=torch.randint(2, V - 1, (B, L), generator=g),
                text_lengths=torch.full((B,), L, dtype=torch.long))


PMC_FILE = os.path.join(ROOT, "profiles", "pmc_conv2_fwd.json")
# every GEMM translation unit and the headers they include (the roofline kernel comes from
# gemm_pipe_conv.hip, or gemm_lds_conv.hip with EA_GEMM_PIPE=0)
GEMM_SOURCES = [os.path.join(ROOT, "espnet-1_amd", "csrc", f)
                for f in ("gemm.hip", "gemm_kern.h", "gemm_pipe.hip", "gemm_pipe_conv.hip", "gemm_lds.hip",
                          "gemm_lds_conv.hip", "gemm_grouped.hip", "common.h")]


def gemm_src_sha():
    """Hash of the GEMM kernel sources: ties a PMC traffic measurement to the build it ran on."""
    import hashlib
    h = hashlib.sha256()
    for f in GEMM_SOURCES:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def pmc_traffic():
    """HBM bytes per launch of the roofline kernel from the committed PMC pass
    (scripts/gpu_pmc.sh: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate runs, gfx950
    FETCH_SIZE x2 correction applied), with whether it was measured on the GEMM sources of
    this tree (the file records their hash); (None, None, False) if the file is absent."""
    try:
        with open(PMC_FILE) as f:
            d = json.load(f)
        from espnet_amd._lib import GEMM_PIPE
        # measured on these sources AND on the kernel this build reports as the roofline kernel
        kernel = "gemm_pipe<true, true, 1, 256" if GEMM_PIPE else "gemm_bf16_lds<256, 256"
        same = d.get("gemm_src_sha") == gemm_src_sha() and kernel in d.get("kernel", "")
        return int(d["traffic_bytes_per_launch"]), os.path.relpath(PMC_FILE, ROOT), same
    except (OSError, KeyError, ValueError):
        return None, None, False


def cpu_baseline(cfg, seconds_budget=25.0):
    """The oracle (oracle/asr_oracle.py, PyTorch-CPU restatement of the reference step) on
    the host cores: fwd + bwd + clip + Adam on a bounded sample (B=4 of the same shapes)."""
    from oracle.asr_oracle import OracleASR, OracleTrainer
    torch.set_num_threads(min(os.cpu_count() or 1, int(os.environ.get("OMP_NUM_THREADS", "16"))))
    sample = dict(cfg, B=4)
    model_cpu = build(cfg)
    ocfg = dict(vocab_size=cfg["vocab_size"], encoder_conf=cfg["encoder_conf"],
                decoder_conf=cfg["decoder_conf"] or {}, model_conf=cfg["model_conf"])
    ora = OracleASR(ocfg, {k: v.detach() for k, v in model_cpu.state_dict().items()})
    tr = OracleTrainer(ora, cfg["optim"]["lr"], cfg["optim"]["weight_decay"], cfg["warmup_steps"])
    batch = synthetic_batch(sample, 1)
    times = []
    t_start = time.perf_counter()
    while True:
        t0 = time.perf_counter()
        tr.step(batch)
        times.append(time.perf_counter() - t0)
        if time.perf_counter() - t_start > seconds_budget or len(times) >= 6:
            break
    steady = sorted(times[1:] if len(times) > 1 else times)
    t = steady[len(steady) // 2]
    return dict(value=round(sample["B"] / t, 4), unit="utterances/s", cores=torch.get_num_threads(),
                kind="port",
                sample=f"oracle step (fwd+bwd+clip+Adam, dropout 0.1, fp32) at B={sample['B']}, "
                       f"T={cfg['T']}, L={cfg['L']}; median of {len(steady)} steps "
                       f"({t:.2f} s/step)")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)   # median over >= 50 steps
    ap.add_argument("--warmup", type=int, default=10)  # after 10 warm-up steps
    ap.add_argument("--config", default="c3", choices=["c3", "c2", "c5"])
    ap.add_argument("--fp32", action="store_true", help="exact-f32 MFMA instead of bf16 AMP")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--profile-steps", type=int, default=0)
    ap.add_argument("--graph-dp", action="store_true",
                    help="(kept for old command lines) with N > 1 the step incl. its RCCL all-reduces "
                         "is captured as a hipGraph by default")
    ap.add_argument("--eager-dp", action="store_true",
                    help="with N > 1, launch every kernel and collective eagerly instead")
    ap.add_argument("--eager", action="store_true", help="launch every kernel from Python each step "
                    "(default: the step is captured once as a hipGraph and replayed)")
    ap.add_argument("--no-dp-rehearsal", action="store_true",
                    help="at N=1, skip the second timing of the step as one rank of a DP job (a "
                         "world-1 RCCL group with every collective of an N-GPU step)")
    ap.add_argument("--dp-rehearsal-steps", type=int, default=20)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # EA_DIST_BACKEND=gloo rehearses the N > 1 path with several ranks sharing one GPU
    backend = os.environ.get("EA_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local = local % torch.cuda.device_count()
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if backend == "nccl":
            from espnet_amd.train.graph import prepare_nccl_env
            prepare_nccl_env()
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)

    from espnet_amd import hip_ops
    from espnet_amd._lib import GEMM_PIPE
    from espnet_amd.optim.adam import ArenaAdam
    from espnet_amd.schedulers.warmup_lr import WarmupLR
    from espnet_amd.train.distributed import ArenaDataParallel
    from espnet_amd.train.graph import CapturedTrainStep

    if args.config == "c5":
        return run_c5(args, world, rank, dev)
    cfg = _diag_dropout(c3_config() if args.config == "c3" else c2_config())
    amp = not args.fp32
    model = build(cfg)
    model.prepare(dev, amp=amp, seed=1234)
    model.train()
    opt = ArenaAdam(model, lr=cfg["optim"]["lr"], weight_decay=cfg["optim"]["weight_decay"])
    sched = WarmupLR(opt, warmup_steps=cfg["warmup_steps"])
    dp = ArenaDataParallel(model) if world > 1 else None
    host = synthetic_batch(cfg, 1 + rank)  # abs_task.py:1566-1575: each rank its own shard
    batch = {k: v.to(dev) for k, v in host.items()}  # resident in HBM before timing
    maxlens = (cfg["T"], cfg["L"])
    # multi-GPU steps are captured with their RCCL collectives too (tests/test_dp_capture_gpu.py:
    # bit-identical to eager DP); CapturedTrainStep falls back to eager steps if a node's stack
    # cannot capture them
    eager = args.eager or (world > 1 and args.eager_dp)
    runner = CapturedTrainStep(model, opt, sched, grad_clip=5.0, dp=dp, warmup=2, enabled=not eager)

    def step():
        return runner(batch, maxlens)

    def timed(step_fn, steps):
        """Barrier + synchronize on both sides of exactly `steps` steps; per-step HIP events
        on the step's stream.  -> (wall seconds, max over ranks; sorted per-step ms; the last
        step's outputs)."""
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
        t0 = time.perf_counter()
        evs[0].record()
        last = None
        for i in range(steps):
            last = step_fn()
            evs[i + 1].record()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el, sorted(evs[i].elapsed_time(evs[i + 1]) for i in range(steps)), last

    # in-kernel span probe of the dominant GEMM; captured into the graph, so it measures
    # every replay; reset after warmup so only the timed region counts
    probe = hip_ops.KernelProbe(["conv2_gemm"], dev)
    hip_ops.PROBE = probe
    for _ in range(max(args.warmup, 0 if eager else 3)):
        step()
    torch.cuda.synchronize()
    sync_capture_mode(runner, world)
    probe.reset()
    # per-step HIP events on the step's stream (median step time)
    elapsed, step_ms, (loss, stats, weight, gn) = timed(step, args.steps)
    hip_ops.PROBE = None
    step_mode = runner.mode or "eager"
    ms = elapsed / args.steps * 1e3
    utt = cfg["B"] * world * args.steps / elapsed
    conv_ms, n_conv = probe.mean_ms("conv2_gemm")
    # the same launch timed with HIP events on its stream: eager forwards of the subsampling
    # block after the timed region (events cannot sit inside the captured graph)
    ev_probe = hip_ops.EventProbe(["conv2_gemm"])
    hip_ops.PROBE = ev_probe
    with torch.no_grad():
        for i in range(6):
            if i == 1:
                ev_probe.reset()  # first launch warms the eager path
            model.encoder.embed(batch["speech"], 0)
    conv_ev_ms, n_ev = ev_probe.mean_ms("conv2_gemm")
    hip_ops.PROBE = None
    med_ms = step_ms[len(step_ms) // 2]
    B, T = cfg["B"], cfg["T"]
    T1, F1 = (T - 3) // 2 + 1, (80 - 3) // 2 + 1
    T2, F2 = (T1 - 3) // 2 + 1, (F1 - 3) // 2 + 1
    C = cfg["encoder_conf"]["output_size"]
    conv_flop = 2.0 * B * T2 * F2 * C * 9 * C
    dtype = "bf16" if amp else "f32"
    achieved = conv_flop / (conv_ms * 1e-3) / 1e12
    loss_v = float(loss.item())
    traffic, traffic_src, traffic_same = pmc_traffic() if (args.config == "c3" and amp) else (None, None, False)
    rehearsal = None
    if world == 1 and not args.no_dp_rehearsal and args.dp_rehearsal_steps > 0:
        rehearsal = dp_rehearsal(model, opt, sched, batch, maxlens, cfg, eager, args, timed)
    if rank == 0:
        out = {
            "metric": METRIC, "value": round(utt, 3), "unit": "utterances/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": dtype,
            "data": "synthetic (speech ~N(0,1) fbank-shaped, uniform tokens; random-init weights)",
            "config": {"workload": f"{args.config.upper()} " + (
                "Conformer-L (12x512, 8 heads, ff 2048, cnn 31) + 6-layer Transformer decoder, "
                "hybrid CTC/att 0.3/0.7, lsm 0.1, V=5000, T=1000 frames x 80, L=40, dropout 0.1, "
                "Adam+WarmupLR+clip 5" if args.config == "c3" else
                "Conformer-S (6x256, 4 heads, ff 1024), CTC only, V=5000, T=500, L=20"),
                "global_batch": B * world, "seq_len": T, "parallelism": f"dp{world}",
                **({"diag_dropout": float(os.environ["EA_BENCH_DIAG_DROPOUT"])}
                   if "EA_BENCH_DIAG_DROPOUT" in os.environ else {})},
            "model_tflops_per_s": round(cfg["gflop_per_step"] * world / (ms * 1e-3) / 1e3, 2),
            "roofline": {"bound": "mfma", "kernel": ("gemm_pipe" if GEMM_PIPE else "gemm_bf16_lds") +
                         f" bf16 conv2 implicit GEMM (subsampling forward, M={B * T2 * F2} N={C} K={9 * C})",
                         "achieved": round(achieved, 2), "peak": PEAK[dtype], "unit": "TFLOP/s",
                         "frac": round(achieved / PEAK[dtype], 4), "traffic": traffic,
                         "traffic_unit": "bytes/launch (HBM, PMC)", "traffic_source": traffic_src,
                         "traffic_measured_on_this_build": traffic_same,
                         "algorithmic_bytes": int(2 * (B * T1 * F1 * C + C * 9 * C + B * T2 * F2 * C)),
                         "launch_ms": round(conv_ms, 4), "launches": n_conv,
                         "timing": "achieved/frac from the in-kernel probe (first-block start to "
                                   "last-block end, every timed replay); frac_events from HIP "
                                   "events around eager launches on the launch stream",
                         "launch_ms_events": round(conv_ev_ms, 4), "launches_events": n_ev,
                         "frac_events": round(conv_flop / (conv_ev_ms * 1e-3) / 1e12 / PEAK[dtype], 4)},
            "step_mode": step_mode,
            "step_ms_median": round(med_ms, 3),
            "step_ms_p10_p90": [round(step_ms[len(step_ms) // 10], 3), round(step_ms[(9 * len(step_ms)) // 10], 3)],
            "value_median": round(cfg["B"] * world / (med_ms * 1e-3), 3),
            "loss": round(loss_v, 4),
        }
        if rehearsal is not None:
            out["dp_rehearsal"] = rehearsal
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(cfg)
            out["speedup_vs_cpu"] = round(utt / out["cpu_baseline"]["value"], 1)
        emit(out)
    if world > 1:
        dist.destroy_process_group()


def sync_capture_mode(runner, world):
    """After the warm-up (outside any capture): if a capture failed on any rank, every rank
    runs eager steps, so the timed region measures one mode.  Ranks capture on their own
    (train/graph.py: per-rank shape keys, no collective at capture time)."""
    if world <= 1:
        return
    flag = torch.tensor([runner.capture_failed_flag()], dtype=torch.int32, device=torch.cuda.current_device())
    dist.all_reduce(flag)
    if int(flag.item()) > 0:
        runner.force_eager()


def dp_rehearsal(model, opt, sched, batch, maxlens, cfg, eager, args, timed):
    """The per-rank step of an N-GPU job, timed on this one GPU: a world-1 RCCL group and
    ArenaDataParallel(force_collectives=True), so the step issues every collective of an
    N-GPU step (BatchNorm-buffer broadcasts, the packed stats all-reduce, the 64 MiB gradient
    bucket all-reduces from the grad-ready hooks) and flushes the deferred weight-gradient
    GEMMs per bucket as DP does — captured with its collectives like the N > 1 bench.  The
    all-reduces of a world-1 group move no data over xGMI, so this prices the step structure
    (per-bucket flushes, collective launches), not the link time."""
    from espnet_amd.train.distributed import ArenaDataParallel
    from espnet_amd.train.graph import CapturedTrainStep
    own = False
    try:
        if not dist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if "MASTER_PORT" not in os.environ:
                import socket
                with socket.socket() as sk:
                    sk.bind(("127.0.0.1", 0))
                    os.environ["MASTER_PORT"] = str(sk.getsockname()[1])
            from espnet_amd.train.graph import prepare_nccl_env
            prepare_nccl_env()
            dist.init_process_group("nccl", rank=0, world_size=1, device_id=batch["speech"].device)
            own = True
        dp = ArenaDataParallel(model, force_collectives=True)
        runner = CapturedTrainStep(model, opt, sched, grad_clip=5.0, dp=dp, warmup=2, enabled=not eager)
        for _ in range(max(3, args.warmup // 2)):
            runner(batch, maxlens)
        torch.cuda.synchronize()
        el, ms, _ = timed(lambda: runner(batch, maxlens), args.dp_rehearsal_steps)
        runner.graphs.clear()
        return {"what": "this step as one rank of a DP job: world-1 RCCL group, every collective of an "
                        "N-GPU step issued (no xGMI traffic), weight-gradient GEMMs flushed per 64 MiB bucket",
                "step_mode": runner.mode or "eager", "steps": args.dp_rehearsal_steps,
                "ms_per_step": round(el / args.dp_rehearsal_steps * 1e3, 3),
                "step_ms_median": round(ms[len(ms) // 2], 3),
                "value": round(cfg["B"] * args.dp_rehearsal_steps / el, 3), "buckets": len(dp.buckets)}
    except Exception as e:  # reported, never fatal for the N=1 line
        return {"error": f"{type(e).__name__}: {e}"}
    finally:
        if own:
            dist.destroy_process_group()


def run_c5(args, world, rank, dev):
    """C5: bucketed variable-length batches + SpecAug.  One captured hipGraph per bucket
    shape (SpecAug draws on the host like the reference, copied to the device before each
    replay); --eager launches every step.  value = utterances/s over all ranks; frames/s
    and the padding fraction are reported alongside."""
    from espnet_amd.optim.adam import ArenaAdam
    from espnet_amd.schedulers.warmup_lr import WarmupLR
    from espnet_amd.train.distributed import ArenaDataParallel
    from espnet_amd.train.graph import CapturedTrainStep

    cfg = c5_config()
    amp = not args.fp32
    model = build(cfg)
    model.prepare(dev, amp=amp, seed=1234)
    model.train()
    opt = ArenaAdam(model, lr=cfg["optim"]["lr"], weight_decay=cfg["optim"]["weight_decay"])
    sched = WarmupLR(opt, warmup_steps=cfg["warmup_steps"])
    dp = ArenaDataParallel(model) if world > 1 else None
    batches = c5_batches(cfg, rank, world)
    dbatches = []
    for b in batches:  # resident in HBM before timing
        d = {k: (v.to(dev) if isinstance(v, torch.Tensor) else v) for k, v in b.items()}
        dbatches.append(d)
    nb = len(dbatches)
    torch.manual_seed(1234 + rank)  # SpecAug's host draws
    # one hipGraph per bucket shape (B, T, L): SpecAug's draws are made on the host before
    # each replay into a static device buffer (train/graph.py); --eager launches every step
    runner = CapturedTrainStep(model, opt, sched, grad_clip=5.0, dp=dp, warmup=1, enabled=not args.eager)

    def step(i):
        b = dict(dbatches[i % nb])
        maxlens = b.pop("_maxlens")
        lens_host = b.pop("_lens_host")
        return runner(b, maxlens, lens_host=lens_host)

    # every bucket shape is seen twice before timing (one eager step, then the capture)
    warmup = max(args.warmup, 0 if args.eager else 2 * nb)
    for i in range(warmup):
        step(i)
    torch.cuda.synchronize()
    sync_capture_mode(runner, world)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    n_utt = n_frames = n_padded = 0
    t0 = time.perf_counter()
    for i in range(warmup, warmup + args.steps):
        loss, stats, weight, gn = step(i)
        b = dbatches[i % nb]
        n_utt += len(b["_lens_host"])
        n_frames += sum(b["_lens_host"])
        n_padded += len(b["_lens_host"]) * b["_maxlens"][0]
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    tot = torch.tensor([elapsed, n_utt, n_frames, n_padded], dtype=torch.float64, device=dev)
    if world > 1:
        mx = tot[:1].clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        elapsed = float(mx.item())
    _, n_utt, n_frames, n_padded = (float(v) for v in tot.tolist())
    if rank == 0:
        emit({
            "metric": "utterances/sec, Conformer-L + SpecAug, bucketed T~U[200,2000] (C5)",
            "value": round(n_utt / elapsed, 3), "unit": "utterances/s", "n_gpus": world, "steps": args.steps,
            "warmup": warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16" if amp else "f32",
            "data": "synthetic corpus (speech ~N(0,1), T~U[200,2000], L=round(T/25)); random-init weights",
            "config": {"workload": "C5 Conformer-L + 6-layer decoder + SpecAug (conformer8), NumElements "
                                   f"batch_bins {cfg['batch_bins']} per GPU, "
                                   + ("eager steps" if args.eager else "one captured hipGraph per bucket shape"),
                       "global_batch": None, "seq_len": "200-2000", "parallelism": f"dp{world}"},
            "frames_per_s": round(n_frames / elapsed, 1),
            "padding_fraction": round(1.0 - n_frames / n_padded, 4),
            "batches_in_corpus_per_rank": nb, "step_mode": runner.mode or "eager", "loss": round(float(loss.item()), 4),
        })
    if world > 1:
        dist.destroy_process_group()


_JSON_FD = None  # the process's original stdout: the one JSON line goes there


def emit(obj):
    line = (json.dumps(obj) + "\n").encode()
    if _JSON_FD is None:
        sys.stdout.write(line.decode())
        sys.stdout.flush()
    else:
        os.write(_JSON_FD, line)


if __name__ == "__main__":
    # everything else written to stdout — RCCL's version banner when a communicator comes up
    # (the DP rehearsal, N > 1), library chatter — goes to stderr, so stdout carries exactly
    # one JSON line
    sys.stdout.flush()
    _JSON_FD = os.dup(1)
    os.dup2(2, 1)
    main()
