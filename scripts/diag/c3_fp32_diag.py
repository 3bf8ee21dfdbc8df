"""Diagnostic: which C3 B=32 fp32 gradients drift from float64, and does a switch move them.

Runs the float64 oracle once, then the HIP model (fresh from the seed each time) under the
default settings twice and with the deferral / side-stream switches turned off one at a time.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "espnet-1_amd"))

from goldens import is_null_grad, regenerate_sized  # noqa: E402
from test_model_build import build  # noqa: E402
import test_benched_shapes_gpu as T  # noqa: E402
from espnet_amd import hip_ops as ops  # noqa: E402

WATCH = ("decoder.decoders.1.norm3.weight", "decoder.decoders.1.norm3.bias",
         "decoder.decoders.1.feed_forward.w_1.weight", "decoder.decoders.1.feed_forward.w_1.bias",
         "decoder.decoders.1.feed_forward.w_2.weight", "decoder.decoders.1.norm2.weight")


def run(label, x_grads, prev=None):
    cfg, d, m = regenerate_sized("c3_b2", build)
    inp = T._c3_b32_batch()
    T._hip_step(m, inp, amp=False)
    g = {k: p.grad.detach().cpu().clone() for k, p in m.named_parameters()}
    errs = sorted(((T._rel(g[k], x_grads[k]), k) for k in g if not is_null_grad(k)), reverse=True)
    print(f"[{label}] top:", "; ".join(f"{k} {e:.2e}" for e, k in errs[:6]), flush=True)
    print(f"[{label}] watch:", "; ".join(f"{k.split('decoders.')[-1]} {T._rel(g[k], x_grads[k]):.2e}" for k in WATCH),
          flush=True)
    if prev is not None:
        diff = sorted(((T._rel(g[k], prev[k]), k) for k in g if not is_null_grad(k)), reverse=True)
        print(f"[{label}] vs previous run:", "; ".join(f"{k} {e:.2e}" for e, k in diff[:4]), flush=True)
    del m
    torch.cuda.empty_cache()
    return g


def main():
    cfg, d, m = regenerate_sized("c3_b2", build)
    inp = T._c3_b32_batch()
    _, _, x_grads, _, _ = T._exact_c3_b32(cfg, m, inp)
    del m
    g0 = run("default", x_grads)
    run("default again", x_grads, g0)
    ops.DEFER_REDUCE = False
    run("no deferred reductions", x_grads)
    ops.DEFER_REDUCE = True
    ops.REDUCE_SIDE = False
    run("reductions serial", x_grads)
    ops.REDUCE_SIDE = True
    ops.OVERLAP_WGRAD = False
    run("no side stream", x_grads)


if __name__ == "__main__":
    main()
