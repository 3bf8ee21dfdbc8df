"""The drop-in training surface on the CPU (no GPU needed): the YAML / command-line parser
(espnet2/utils/config_argparse.py, tasks/abs_task.py:261-870, tasks/asr.py:216-355) with
the reference's own task tests (test/espnet2/tasks/test_asr.py, test_abs_task.py), the
recipe config egs2/librispeech/asr1/conf/tuning/train_asr_conformer8.yaml (copied as a
fixture), ClassChoices, NestedDictAction, and the data path (datasets, CommonCollateFn,
SequenceIterFactory, Reporter) against reference goldens (oracle/make_goldens.py)."""
import io
import json
import os

import numpy as np
import pytest
import torch

from goldens import GOLDEN, load

CONFORMER8 = os.path.join(GOLDEN, "train_asr_conformer8.yaml")


def _task():
    from espnet_amd.tasks.asr import ASRTask
    return ASRTask


# --------------------------------------------------------------------- reference task tests
def test_add_arguments():
    _task().get_parser()


def test_add_arguments_help():
    with pytest.raises(SystemExit):
        _task().get_parser().parse_args(["--help"])


def test_main_help():
    with pytest.raises(SystemExit):
        _task().main(cmd=["--help"])


def test_main_print_config(capsys):
    with pytest.raises(SystemExit):
        _task().main(cmd=["--print_config"])
    assert "encoder_conf" in capsys.readouterr().out


def test_main_with_no_args():
    with pytest.raises(SystemExit):
        _task().main(cmd=[])


def test_print_config_and_load_it(tmp_path):
    f = tmp_path / "config.yaml"
    with f.open("w") as fh:
        _task().print_config(fh)
    args = _task().get_parser().parse_args(["--config", str(f)])
    assert args.optim == "adadelta" and args.batch_type == "folded"  # the reference's defaults


# --------------------------------------------------------------------- recipe config
def test_conformer8_recipe_config_builds_c3():
    """The reference recipe YAML parses unchanged and builds BASELINE's C3 model (116.15 M
    parameters, egs2/librispeech/asr1/README.md:475) with input_size 80 (no frontend)."""
    T = _task()
    args = T.get_parser().parse_args(["--config", CONFORMER8, "--input_size", "80", "--output_dir", "x",
                                      "--token_list", "t"])
    T.normalize_args(args)
    assert args.patience is None and args.init is None  # "none" strings in the YAML
    assert args.optim == "adam" and args.optim_conf == {"lr": 0.0025, "weight_decay": 1e-06}
    assert args.scheduler == "warmuplr" and args.scheduler_conf == {"warmup_steps": 40000}
    assert args.accum_grad == 4 and args.use_amp is True and args.batch_type == "numel"
    assert args.best_model_criterion == [["valid", "acc", "max"]]
    args.token_list = ["<blank>", "<unk>"] + [f"t{i}" for i in range(4997)] + ["<sos/eos>"]
    torch.manual_seed(0)
    m = T.build_model(args)
    assert sum(p.numel() for p in m.parameters()) == 116146960
    assert m.specaug is not None and m.frontend is None and type(m.encoder).__name__ == "ConformerEncoder"


def test_command_line_overrides_config():
    args = _task().get_parser().parse_args(["--config", CONFORMER8, "--max_epoch", "3", "--encoder_conf",
                                            "num_blocks=2", "--optim_conf", "lr=0.1"])
    assert args.max_epoch == 3
    # NestedDictAction updates the dict the config set (nested_dict_action.py:68-90)
    assert args.encoder_conf["num_blocks"] == 2 and args.encoder_conf["output_size"] == 512
    assert args.optim_conf == {"lr": 0.1, "weight_decay": 1e-06}


def test_config_unknown_key_is_an_error(tmp_path):
    f = tmp_path / "bad.yaml"
    f.write_text("no_such_option: 1\n")
    with pytest.raises(SystemExit):
        _task().get_parser().parse_args(["--config", str(f)])


def test_nested_dict_action_syntaxes():
    import argparse
    from espnet_amd.utils.nested_dict_action import NestedDictAction
    def parse(*a):  # a fresh parser per call: the dict form updates the default in place, as the reference's
        p = argparse.ArgumentParser()
        p.add_argument("--conf", action=NestedDictAction, default={"a": 4})
        return p.parse_args(list(a)).conf
    assert parse("--conf", "a=3", "--conf", "c=4") == {"a": 3, "c": 4}
    assert parse("--conf", "c.d=4") == {"a": 4, "c": {"d": 4}}
    assert parse("--conf", "c.d=4", "--conf", "c=2") == {"a": 4, "c": 2}
    assert parse("--conf", "{d: 5, e: 9}") == {"a": 4, "d": 5, "e": 9}
    assert parse("--conf", "{'f': True}") == {"a": 4, "f": True}


def test_class_choices_type_check_and_errors():
    from espnet_amd.train.class_choices import ClassChoices
    from espnet_amd.tasks.asr import encoder_choices
    with pytest.raises(ValueError):
        ClassChoices("x", dict(a=int), type_check=str)
    with pytest.raises(ValueError):
        ClassChoices("x", dict(none=int))
    with pytest.raises(ValueError):
        encoder_choices.get_class("branchformer")
    assert encoder_choices.get_class("Transformer").__name__ == "TransformerEncoder"


# --------------------------------------------------------------------- data path
def test_datasets_collate_and_sharding(tmp_path):
    from espnet_amd.fileio.datasets import ESPnetDataset
    from espnet_amd.train.collate_fn import CommonCollateFn
    (tmp_path / "shape").write_text("a 10,80\nb 7,80\nc 12,80\n")
    (tmp_path / "tshape").write_text("a 4\nb 3\nc 5\n")
    (tmp_path / "text").write_text("a 5 6 7 8\nb 9 10 11\nc 1 2 3 4 5\n")
    ds = ESPnetDataset([(str(tmp_path / "shape"), "speech", "rand_float"),
                        (str(tmp_path / "text"), "text", "text_int"),
                        (str(tmp_path / "tshape"), "tok", "rand_int_2_9")])
    uid, d = ds["b"]
    assert d["speech"].shape == (7, 80) and d["speech"].dtype == np.float32
    assert d["text"].tolist() == [9, 10, 11] and d["text"].dtype == np.int64
    assert d["tok"].shape == (3,) and (2 <= d["tok"]).all() and (d["tok"] < 9).all()
    ids, batch = CommonCollateFn(float_pad_value=0.0, int_pad_value=-1)([ds["a"], ds["b"], ds["c"]])
    assert ids == ["a", "b", "c"]
    assert batch["speech"].shape == (3, 12, 80) and batch["speech_lengths"].tolist() == [10, 7, 12]
    assert batch["text"][1].tolist() == [9, 10, 11, -1, -1] and batch["text_lengths"].tolist() == [4, 3, 5]
    assert float(batch["speech"][1, 7:].abs().sum()) == 0.0
    with pytest.raises(NotImplementedError):
        ESPnetDataset([(str(tmp_path / "shape"), "speech", "kaldi_ark")])


def test_sequence_iter_factory_matches_reference():
    from espnet_amd.iterators.sequence_iter_factory import SequenceIterFactory
    cfg, d = load("iterfactory")
    batches = [tuple(b) for b in cfg["batches"]]
    for key, kw in cfg["cases"].items():
        f = SequenceIterFactory(dataset=None, batches=list(batches), seed=cfg["seed"], **kw)
        for epoch in range(1, 6):
            got = [list(b) for b in f.batches_for_epoch(epoch)]
            assert got == json.loads(str(d[f"{key}.e{epoch}"])), (key, epoch)


def test_reporter_matches_reference():
    from espnet_amd.train.reporter import Reporter
    _, d = load("reporter")
    seq = [({"loss": 3.0, "acc": 0.5}, 4, {"lr": 0.1}), ({"loss": float("nan"), "acc": 0.25}, 2, {"lr": 0.2}),
           ({"loss": 1.0, "acc": None}, 3, {}), ({"loss": 2.0, "acc": 0.75, "late": 9.0}, 1, {"lr": 0.4}),
           ({"loss": float("inf"), "acc": 1.0, "late": 1.0}, 5, {"lr": 0.5})]
    rep = Reporter()
    msgs = []
    for e in (1, 2, 3):
        rep.set_epoch(e)
        with rep.observe("train") as sub:
            for st, w, un in seq:
                # device tensors for some values: the lazy path must aggregate identically
                sub.register({k: (None if v is None else (torch.tensor([v * e]) if k == "loss" else v * e))
                              for k, v in st.items()}, torch.tensor([w]) if w % 2 else w)
                if un:
                    sub.register(un)
                sub.next()
                msgs.append(sub.log_message(-2))
        with rep.observe("valid") as sub:
            sub.register({"loss": float(4 - e) if e != 2 else 5.0, "acc": 0.1 * e}, 2)
            sub.next()
    assert msgs == json.loads(str(d["msgs"]))
    for k, v in d.items():
        if k.startswith("e") and k[1].isdigit():
            e, key, k2 = k.split(".", 2)
            got = rep.stats[int(e[1:])][key][k2]
            np.testing.assert_equal(got, float(v), err_msg=k)
    assert rep.sort_epochs("valid", "loss", "min") == d["sort_valid_loss_min"].tolist()
    assert rep.get_best_epoch("train", "acc", "max") == int(d["best_train_acc_max"])
    assert rep.check_early_stopping(0, "valid", "loss", "min") == bool(d["early_stop_p0"])
    assert rep.check_early_stopping(1, "valid", "loss", "min") == bool(d["early_stop_p1"])
