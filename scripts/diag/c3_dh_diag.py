"""Diagnostic: the decoder FFN hidden gradient dh of layer 1 at C3 B=32 fp32, HIP vs float64,
per (utterance, position) row."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "espnet-1_amd"))

from goldens import regenerate_sized  # noqa: E402
from test_model_build import build  # noqa: E402
import test_benched_shapes_gpu as T  # noqa: E402
from espnet_amd import hip_ops as ops  # noqa: E402
import oracle.asr_oracle as OA  # noqa: E402

LAYERS = (0, 1, 2, 3)


def main():
    cfg, d, m = regenerate_sized("c3_b2", build)
    inp = T._c3_b32_batch()
    # oracle: hooks on the w_1 outputs (pre-ReLU) of the watched layers
    store = {}
    orig_ffn = OA.ffn

    def ffn(P, name, x, act, p_drop, training):
        h = OA.linear(P, name + ".w_1", x)
        if name.startswith("decoder.decoders."):
            l = int(name.split(".")[2])
            if l in LAYERS:
                store[("h", l)] = h.detach().clone()
                h.register_hook(lambda g, l=l: store.__setitem__(("dh", l), g.detach().clone()))
        return OA.linear(P, name + ".w_2", OA.drop(act(h), p_drop, training))

    OA.ffn = ffn
    torch.set_num_threads(16)
    ora = OA.OracleASR(cfg, {k: v.detach() for k, v in m.state_dict().items()}, dtype=torch.float64)
    loss, _, _ = ora(**inp)
    loss.backward()
    OA.ffn = orig_ffn
    # HIP: record the column-sum input of each watched layer's w_1 bias gradient (= dh)
    m.prepare(T.DEV, amp=False)
    m.train()
    b = m.decoder._b
    want = {b.g(f"decoders.{l}.feed_forward.w_1.bias").data_ptr(): l for l in LAYERS}
    got = {}
    orig_colsum = ops.colsum

    def colsum(x, out, *a, **k):
        if out.data_ptr() in want:
            got[want[out.data_ptr()]] = x.detach().clone()
        return orig_colsum(x, out, *a, **k)

    ops.colsum = colsum
    import espnet_amd.layers.decoder as D
    D.ops.colsum = colsum
    loss_h, _, _ = m(**inp)
    loss_h.backward()
    torch.cuda.synchronize()
    ops.colsum = orig_colsum
    print(f"loss hip {loss_h.item():.8f} f64 {loss.item():.8f}")
    B, L = inp["text"].shape[0], int(inp["text_lengths"].max()) + 1
    for l in LAYERS:
        if l not in got or ("dh", l) not in store:
            print(f"layer {l}: missing (hip {l in got}, oracle {('dh', l) in store})")
            continue
        dh_h = got[l].double().cpu().view(B, L, -1)
        dh_x = store[("dh", l)].view(B, L, -1)
        h_x = store[("h", l)].view(B, L, -1)
        # the oracle hook sees the gradient before the ReLU mask; apply it
        dh_x = dh_x * (h_x > 0)
        tot = T._rel(dh_h, dh_x)
        err = (dh_h - dh_x).norm(dim=-1)
        ref = dh_x.norm(dim=-1)
        worst = torch.argsort(err.flatten(), descending=True)[:8]
        print(f"layer {l}: dh rel L2 {tot:.3e}; column-sum rel {T._rel(dh_h.sum((0, 1)), dh_x.sum((0, 1))):.3e}")
        for i in worst.tolist():
            bb, ll = divmod(i, L)
            print(f"   utt {bb:2d} pos {ll:2d} (len {int(inp['text_lengths'][bb]) + 1}): |err| {err[bb, ll]:.3e} "
                  f"|ref| {ref[bb, ll]:.3e}")
        nz = (h_x == 0).sum().item()
        print(f"   exact zero pre-activations in the oracle: {nz}; |h| < 1e-6: {(h_x.abs() < 1e-6).sum().item()}")


if __name__ == "__main__":
    main()
