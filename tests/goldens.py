"""Helpers to read the golden fixtures written by oracle/make_goldens.py."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"))  # allow_pickle=False (default)
    d = {k: z[k] for k in z.files}
    cfg = json.loads(str(d.pop("cfg"))) if "cfg" in d else None
    return cfg, d


def section(d, prefix):
    n = len(prefix) + 1
    return {k[n:]: v for k, v in d.items() if k.startswith(prefix + ".")}


# Parameters whose exact gradient is identically zero: a key bias adds the same constant to
# every score of a query row (softmax is shift-invariant, attention.py:63-93), and the
# depthwise-conv bias is removed again by the BatchNorm that follows it (convolution.py:
# 70-75, batch statistics in training).  Their fp32 gradients are rounding noise (|g| ~
# 1e-10..1e-5), so they are checked for smallness against the sibling weight's gradient
# instead of element-wise.
NULL_GRAD_SUFFIXES = ("self_attn.linear_k.bias", "src_attn.linear_k.bias", "depthwise_conv.bias")


def is_null_grad(name):
    return name.endswith(NULL_GRAD_SUFFIXES)


def sibling_weight(name):
    return name[: -len("bias")] + "weight"


def assert_grad_close(mine, ref, name, rtol=2e-4, scale_tol=1e-3, atol=0.0):
    """fp32 gradient parity: |mine - ref| <= rtol*|ref| + scale_tol*max|ref| element-wise.
    The scale term is the fp32 summation-order noise of a deep backward (reduction over
    B*T' rows in a different order than ATen's): relative to the tensor's largest entry,
    not to each (possibly near-zero) element."""
    import numpy as np
    mine = np.asarray(mine, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    scale = float(np.abs(ref).max()) if ref.size else 0.0
    np.testing.assert_allclose(mine, ref, rtol=rtol, atol=max(atol, scale_tol * scale) + 1e-12, err_msg=name)


def perturb_norms(model, gen):
    """The same perturbation oracle/make_goldens.py applies before a capture (LayerNorm /
    BatchNorm affine parameters and BN running stats made non-trivial), in the same
    named_parameters / named_buffers order."""
    import torch
    with torch.no_grad():
        for name, p in model.named_parameters():
            if "norm" in name:
                p.add_(0.1 * torch.randn(p.shape, generator=gen))
        for name, b in model.named_buffers():
            if name.endswith("running_mean"):
                b.copy_(0.1 * torch.randn(b.shape, generator=gen))
            elif name.endswith("running_var"):
                b.copy_(1.0 + 0.2 * torch.rand(b.shape, generator=gen))


def regenerate_sized(name, build):
    """Rebuild the weights of a BASELINE-sized golden (oracle/make_goldens.py capture_sized)
    from its seed on the CPU and check them against the stored per-tensor sums."""
    import numpy as np
    import torch
    cfg, d = load(name)
    torch.manual_seed(cfg["seed"])
    m = build(cfg)
    perturb_norms(m, torch.Generator().manual_seed(1000 + cfg["seed"]))
    sd = m.state_dict()
    sums = section(d, "wsum")
    if cfg["model_conf"]["ctc_weight"] == 1.0:
        sums = {k: v for k, v in sums.items() if not k.startswith("decoder.")}
    assert list(sd) == list(sums), "state_dict layout differs from the reference's"
    for k, v in sums.items():
        np.testing.assert_allclose(sd[k].double().sum().item(), float(v), rtol=1e-12, atol=1e-12, err_msg=k)
    return cfg, d, m
