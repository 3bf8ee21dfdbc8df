"""Timeline of the last complete training step in a rocprofv3 DB: wall time between the
last two adam_kernel ends, busy time (union of kernel intervals), idle gaps, and per-
category kernel time. usage: python scripts/timeline.py DB"""
import collections
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, start, end, stream_id, queue_id from kernels order by start").fetchall()
ad = [r for r in rows if "adam_kernel" in r[0]]
t0, t1 = ad[-2][2], ad[-1][2]
step = [r for r in rows if r[1] >= t0 and r[2] <= t1]
wall = (t1 - t0) / 1e3
iv = sorted((r[1], r[2]) for r in step)
busy, cs, ce = 0, None, None
gaps = []
for s, e in iv:
    if cs is None:
        cs, ce = s, e
    elif s > ce:
        busy += ce - cs
        gaps.append(s - ce)
        cs, ce = s, e
    else:
        ce = max(ce, e)
busy += ce - cs
print(f"step wall {wall:.1f} us, kernels {len(step)}, busy(union) {busy/1e3:.1f} us, idle {wall - busy/1e3:.1f} us,"
      f" gaps {len(gaps)} (mean {sum(gaps)/max(1,len(gaps))/1e3:.2f} us)")
print("queues:", collections.Counter(r[4] for r in step))
cat = collections.defaultdict(lambda: [0, 0])
def catname(n):
    for k in ("gemm_bf16_lds", "splitk_reduce", "reduce_partials", "attn_bwd", "attn_fwd", "ln_", "colsum", "bn_",
              "dwconv", "adam", "ctc", "lsm", "drop", "glu", "conv1", "embed", "rocclr", "Fill", "sqnorm", "mha", "softmax"):
        if k in n:
            return k
    return n[:60]
for r in step:
    k = catname(r[0]); cat[k][0] += r[2] - r[1]; cat[k][1] += 1
tot = sum(v[0] for v in cat.values())
print(f"sum of kernel durations {tot/1e3:.1f} us")
for k, (d, n) in sorted(cat.items(), key=lambda x: -x[1][0]):
    print(f"{d/1e3:9.1f} us {n:5d}  {k}")
