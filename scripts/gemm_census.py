"""GEMM census of one C3 training step: every ea_gemm call (shape, layouts, epilogue) timed
with HIP events (serial: EA_OVERLAP_WGRAD=0), grouped, with TFLOP/s and share of the step.

    EA_OVERLAP_WGRAD=0 python scripts/gemm_census.py [c3|c2]
"""
import collections
import os
import sys

os.environ.setdefault("EA_OVERLAP_WGRAD", "0")
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "espnet-1_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from espnet_amd import hip_ops as ops  # noqa: E402
from espnet_amd.optim.adam import ArenaAdam  # noqa: E402
from espnet_amd.schedulers.warmup_lr import WarmupLR  # noqa: E402
from espnet_amd.train.trainer import Trainer  # noqa: E402

cfg = bench.c3_config() if (len(sys.argv) < 2 or sys.argv[1] == "c3") else bench.c2_config()
dev = torch.device("cuda", 0)
model = bench.build(cfg)
model.prepare(dev, amp=True, seed=1234)
model.train()
opt = ArenaAdam(model, lr=cfg["optim"]["lr"], weight_decay=cfg["optim"]["weight_decay"])
sched = WarmupLR(opt, warmup_steps=cfg["warmup_steps"])
host = bench.synthetic_batch(cfg, 1)
batch = {k: v.to(dev) for k, v in host.items()}

records = []
_orig = ops.gemm


def timed_gemm(A, B, C, *, M, N, K, a_kmajor, b_kmajor, batch=1, nh=1, epi=None, **kw):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    r = _orig(A, B, C, M=M, N=N, K=K, a_kmajor=a_kmajor, b_kmajor=b_kmajor, batch=batch, nh=nh, epi=epi, **kw)
    e1.record()
    kind = epi.kind if epi is not None else 0
    drop = epi.drop_p > 0 if epi is not None else False
    records.append(((M, N, K, int(a_kmajor), int(b_kmajor), batch * nh, kind, drop, str(C.dtype)[6:]), e0, e1))
    return r


ops.gemm = timed_gemm
_orig_flush = ops.WgradQueue.flush


def timed_flush(self):
    if not self.items:
        return
    n, K0 = len(self.items), max(it[0] for it in self.items)
    f = sum(2.0 * it[4] * it[5] * it[0] for it in self.items)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    _orig_flush(self)
    e1.record()
    records.append((("grouped", n, K0, f), e0, e1))


ops.WgradQueue.flush = timed_flush
for _ in range(2):
    Trainer.train_one_step(model, batch, opt, sched, grad_clip=5.0)
torch.cuda.synchronize()
records.clear()
step_ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
step_ev[0].record()
Trainer.train_one_step(model, batch, opt, sched, grad_clip=5.0)
step_ev[1].record()
torch.cuda.synchronize()
step_ms = step_ev[0].elapsed_time(step_ev[1])
agg = collections.defaultdict(lambda: [0, 0.0])
for key, e0, e1 in records:
    agg[key][0] += 1
    agg[key][1] += e0.elapsed_time(e1)
tot = sum(v[1] for v in agg.values())
flops = 0.0
print(f"step (serial wgrad) {step_ms:.3f} ms; GEMM total {tot:.3f} ms over {len(records)} calls")
print(f"{'M':>7} {'N':>5} {'K':>6} ak bk  z epi drop out   calls   ms/step    us/call  TF/s  %step")
for key, (n, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    if key[0] == "grouped":
        _, nprob, K0, f = key
        flops += f * n
        print(f"grouped wgrad: {nprob} problems (max K {K0}) x{n}: {ms:9.3f} ms/step  {f * n / (ms * 1e-3) / 1e12:6.0f} TF/s"
              f"  {100 * ms / step_ms:5.1f}%")
        continue
    M, N, K, ak, bk, z, kind, drop, od = key
    f = 2.0 * M * N * K * z * n
    flops += f
    print(f"{M:7d} {N:5d} {K:6d} {ak:2d} {bk:2d} {z:3d} {kind:3d} {int(drop):4d} {od:5s} {n:5d} {ms:9.3f} "
          f"{ms / n * 1e3:10.1f} {f / (ms * 1e-3) / 1e12:6.0f} {100 * ms / step_ms:5.1f}")
print(f"GEMM flops {flops / 1e9:.1f} GF, {flops / (tot * 1e-3) / 1e12:.0f} TF/s average")
