"""Run-to-run determinism of the single-process training step (no DP hooks): the DP tests'
tiny model, 6 steps from the same initial weights, N times in one process, every run's final
arena compared bit for bit with the first.  usage: sp_determinism.py [N]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import torch  # noqa: E402

import test_dp_capture_gpu as C  # noqa: E402
import test_dp_ragged_gpu as R  # noqa: E402


def one():
    from espnet_amd.train.trainer import Trainer
    _, m, opt, sched = C._setup(amp=True, dropout=0.1)
    for b in R._global_batches(6):
        Trainer.train_one_step(m, {k: v.to("cuda:0") for k, v in b.items()}, opt, sched, grad_clip=5.0)
    torch.cuda.synchronize()
    return m.arena.data.cpu().clone()


def one_c3(state={}):
    """The bench's C3 model (B=32, T=1000), 3 eager steps from the same initial weights."""
    import bench
    from espnet_amd.optim.adam import ArenaAdam
    from espnet_amd.schedulers.warmup_lr import WarmupLR
    from espnet_amd.train.trainer import Trainer
    cfg = bench.c3_config()
    if "w0" not in state:
        m = bench.build(cfg)
        state["sd"] = {k: v.clone() for k, v in m.state_dict().items()}
        state["w0"] = True
    m = bench.build(cfg)
    m.load_state_dict(state["sd"])
    m.prepare(torch.device("cuda", 0), amp=True, seed=1234)
    m.train()
    opt = ArenaAdam(m, lr=0.002, weight_decay=1e-6)
    sched = WarmupLR(opt, warmup_steps=25000)
    for s in range(3):
        b = bench.synthetic_batch(cfg, s)
        Trainer.train_one_step(m, {k: v.to("cuda:0") for k, v in b.items()}, opt, sched, grad_clip=5.0)
    torch.cuda.synchronize()
    return m.arena.data.cpu().clone()


def main():
    C._paths() if hasattr(C, "_paths") else None
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    global one
    if len(sys.argv) > 2 and sys.argv[2] == "c3":
        one = one_c3
    ref = one()
    bad = 0
    for i in range(1, n):
        w = one()
        if not torch.equal(w, ref):
            bad += 1
            d = (w - ref).abs()
            print(f"run {i}: {int((d > 0).sum())} elements differ, max {float(d.max()):.3g}", flush=True)
    print(f"single process: {bad} of {n - 1} runs differ from the first", flush=True)


if __name__ == "__main__":
    main()
