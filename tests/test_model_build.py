"""CPU checks of the host-side mirror: the HIP-backed modules expose the reference's
state_dict layout and initialise identically under the same seed (no GPU needed)."""
import pytest
import torch

from goldens import load, section


def build(cfg):
    from espnet_amd.tasks.asr import build_model
    V = cfg["vocab_size"]
    tok = ["<blank>", "<unk>"] + [f"t{i}" for i in range(V - 3)] + ["<sos/eos>"]
    args = dict(token_list=tok, input_size=cfg["input_size"], encoder=cfg["encoder"],
                encoder_conf=cfg["encoder_conf"], decoder=cfg.get("decoder"),
                decoder_conf=cfg.get("decoder_conf", {}), model_conf=cfg["model_conf"],
                normalize="utterance_mvn")
    return build_model(args)


@pytest.mark.parametrize("name", ["tiny_hybrid", "tiny_ctc", "medium_hybrid", "c1_tiny"])
def test_state_dict_layout_and_init(name):
    cfg, d = load(name)
    torch.manual_seed(0)
    m = build(cfg)
    ref = section(d, "w")
    sd = m.state_dict()
    if cfg["model_conf"]["ctc_weight"] == 1.0:
        ref = {k: v for k, v in ref.items() if not k.startswith("decoder.")}
    assert list(sd.keys()) == list(ref.keys())
    for k, v in ref.items():
        assert tuple(sd[k].shape) == tuple(v.shape), k
        if "norm" in k or "running" in k or "num_batches" in k:
            continue  # the goldens perturb norm params / BN stats on purpose
        torch.testing.assert_close(sd[k].float(), torch.from_numpy(v).float(), rtol=0, atol=0,
                                   msg=f"init differs for {k}")


def test_unsupported_options_raise():
    cfg, _ = load("tiny_hybrid")
    bad = dict(cfg)
    bad["encoder_conf"] = dict(cfg["encoder_conf"], input_layer="linear")
    with pytest.raises(NotImplementedError):
        build(bad)
    bad["encoder_conf"] = dict(cfg["encoder_conf"], rel_pos_type="nope")
    with pytest.raises(ValueError):
        build(bad)


def test_header_symbols_exported():
    """The C-ABI library loads and exports every symbol include/espnet_amd.h declares."""
    import ctypes
    import os
    from espnet_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("library not built")
    dll = ctypes.CDLL(_lib.LIB_PATH)
    protos = _lib.parse_header()
    assert len(protos) >= 30
    for name in protos:
        assert hasattr(dll, name), name
    # the entry points that do not return int (the diagnostic allocator's pair)
    import re
    src = re.sub(r"/\*.*?\*/", "", open(_lib.HEADER).read(), flags=re.S)
    others = re.findall(r"\bvoid\s*\*?\s*(ea_\w+)\s*\(", src)
    assert others
    for name in others:
        assert hasattr(dll, name), name
