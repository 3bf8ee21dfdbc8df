"""SpecAug (C5): the oracle restatement and the HIP kernel against the
reference's own SpecAug run under fixed torch seeds (tests/golden/specaug.npz, captured by
oracle/make_goldens.py from espnet2/asr/specaug/specaug.py), plus the NumElementsBatchSampler
batch lists (tests/golden/sampler.npz).

Tolerances: mask spans and warp points are drawn with the reference's torch.randint calls on
the CPU generator, so WHICH frames/bins are zeroed and where the warp splits are exact; the
warped values come from a bicubic resample whose weight arithmetic ATen's CPU kernel rounds
differently from a plain restatement (measured <= 1.7e-5 absolute at |x| <= 5), so warped
values are compared with atol 5e-5, rtol 1e-5; unwarped / masked values are bit-exact.
"""
import json
import os
import sys

import numpy as np
import pytest
import torch

from goldens import load

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _cases():
    cfg, d = load("specaug")
    return cfg, d


@pytest.mark.parametrize("case", ["eq", "ragged", "eq_long", "fixed"])
def test_oracle_specaug_matches_reference(case):
    from oracle.asr_oracle import specaug
    cfg, d = _cases()
    conf_name, lens, Fd, seed = cfg["cases"][case]
    torch.manual_seed(seed)
    y = specaug(torch.from_numpy(d[f"{case}.x"]), torch.from_numpy(d[f"{case}.lens"]), cfg["confs"][conf_name])
    assert np.array_equal(y.numpy(), d[f"{case}.y"])


@pytest.mark.parametrize("case", ["eq", "ragged", "eq_long", "fixed"])
def test_specaug_draws_match_reference(case):
    """The product module's host draws (no GPU needed) reproduce the reference's masks
    exactly: every bin the reference zeroed (and that was non-zero in its input) is inside
    one of our drawn spans, and vice versa."""
    from espnet_amd.asr.specaug import SpecAug
    cfg, d = _cases()
    conf_name, lens, Fd, seed = cfg["cases"][case]
    conf = cfg["confs"][conf_name]
    x, y = d[f"{case}.x"], d[f"{case}.y"]
    B, T, _ = x.shape
    torch.manual_seed(seed)
    warp, per_utt, fm, tm = SpecAug(**conf).draw(B, T, Fd, [int(v) for v in lens])
    assert per_utt == int(len(set(lens)) > 1 and conf.get("apply_time_warp", True))
    zero = np.zeros_like(y, dtype=bool)
    for b in range(B):
        for (p, w) in (fm[b].tolist() if fm is not None else []):
            zero[b, :, p:p + w] = True
        for (p, w) in (tm[b].tolist() if tm is not None else []):
            zero[b, p:p + w, :] = True
    assert (y[zero] == 0).all()
    # outside the spans the reference output is non-zero wherever its input frame was valid
    valid = np.zeros_like(zero)
    for b, le in enumerate(lens):
        valid[b, :le] = True
    assert (y[valid & ~zero] != 0).mean() > 0.999


def test_sampler_matches_reference(tmp_path):
    from espnet_amd.samplers.num_elements_batch_sampler import NumElementsBatchSampler
    cfg, d = load("sampler")
    Ts = d["T"]
    sp, tx = tmp_path / "speech_shape", tmp_path / "text_shape"
    sp.write_text("".join(f"utt{i:03d} {t},80\n" for i, t in enumerate(Ts)))
    tx.write_text("".join(f"utt{i:03d} {max(1, round(t / 25))}\n" for i, t in enumerate(Ts)))
    built = cfg.pop("built")
    for key, kw in cfg.items():
        kw = dict(kw)
        kw["shape_files"] = [str(sp), str(tx)][: kw["shape_files"]]
        s = NumElementsBatchSampler(**kw)
        flat = [int(k[3:]) for b in s for k in b]
        sizes = [len(b) for b in s]
        assert flat == d[f"{key}.flat"].tolist(), key
        assert sizes == d[f"{key}.sizes"].tolist(), key
    # every batch type through build_batch_sampler (incl. a category file)
    from espnet_amd.samplers.batch_samplers import build_batch_sampler
    cat = tmp_path / "utt2category"
    cat.write_text("".join(f"utt{i:03d} {'a' if i % 3 else 'b'}\n" for i in range(len(Ts))))
    for key, kw in built.items():
        kw = dict(kw)
        kw["shape_files"] = [str(sp), str(tx)][: kw["shape_files"]]
        if "utt2category_file" in kw:
            kw["utt2category_file"] = str(cat)
        s = build_batch_sampler(**kw)
        assert [int(k[3:]) for b in s for k in b] == d[f"{key}.flat"].tolist(), key
        assert [len(b) for b in s] == d[f"{key}.sizes"].tolist(), key
        assert s.generate(0) == list(s)
    # in-memory shapes give the same batches as the shape files
    mem = NumElementsBatchSampler(400000, utt2shapes=[{f"utt{i:03d}": [int(t), 80] for i, t in enumerate(Ts)}])
    assert [int(k[3:]) for b in mem for k in b] == d["default.flat"].tolist()


def test_specaug_constructor_errors():
    from espnet_amd.asr.specaug import SpecAug
    with pytest.raises(ValueError):
        SpecAug(apply_time_warp=False, apply_freq_mask=False, apply_time_mask=False)
    with pytest.raises(ValueError):
        SpecAug(time_mask_width_range=(0, 10), time_mask_width_ratio_range=(0.0, 0.05))
    with pytest.raises(ValueError):
        SpecAug(apply_time_mask=True)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["eq", "ragged", "eq_long", "fixed"])
def test_specaug_hip_matches_reference(case):
    from espnet_amd.asr.specaug import SpecAug
    cfg, d = _cases()
    conf_name, lens, Fd, seed = cfg["cases"][case]
    x = torch.from_numpy(d[f"{case}.x"]).cuda()
    xl = torch.from_numpy(d[f"{case}.lens"]).cuda()
    torch.manual_seed(seed)
    y, yl = SpecAug(**cfg["confs"][conf_name])(x, xl, lens_host=[int(v) for v in lens])
    torch.cuda.synchronize()
    ref = d[f"{case}.y"]
    got = y.cpu().numpy()
    assert ((ref == 0) == (got == 0)).mean() > 0.9999
    np.testing.assert_allclose(got, ref, atol=5e-5, rtol=1e-5)
    if not cfg["confs"][conf_name].get("apply_time_warp", True):
        assert np.array_equal(got, ref)
    assert yl is xl
