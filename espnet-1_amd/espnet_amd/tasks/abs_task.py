"""AbsTask — the command-line / YAML training entry of espnet2/tasks/abs_task.py:
get_parser (:261-870, the same option names, types and defaults), print_config
(:1017-1024), main (:1026-1094: one process, or one spawned worker per GPU) and
main_worker (:1097-1357: distributed init over RCCL, seed, build model / optimizer /
scheduler, config.yaml, iterator factories, Trainer.run).

MI355X specifics: the model is laid into the flat parameter arena on its GPU
(model.prepare; --use_amp selects bf16 MFMA operands exactly where the reference's
autocast does), the optimizer is the arena Adam (one kernel for clip + Adam + the bf16
shadow), and the step is captured as a hipGraph per batch shape (train/trainer.py).
Options that only exist for other products or cluster launchers are accepted by the
parser (configs stay loadable) and rejected with NotImplementedError when set to a
non-default value.
"""
from __future__ import annotations

import argparse
import copy
import inspect
import logging
import os
import sys
from pathlib import Path
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import yaml

from ..fileio.datasets import ESPnetDataset
from ..iterators.sequence_iter_factory import SequenceIterFactory
from ..samplers.batch_samplers import BATCH_TYPES, build_batch_sampler
from ..train.distributed_utils import DistributedOption, free_port, resolve_distributed_mode
from ..train.trainer import Trainer
from ..utils.config_argparse import ArgumentParser
from ..utils.nested_dict_action import NestedDictAction
from ..utils.types import (humanfriendly_parse_size_or_none, int_or_none, parse_size, str2bool, str2triple_str,
                           str_or_int, str_or_none)

# abs_task.py:79-120 registries: the names the reference accepts; the build runs "adam"
# (the arena Adam) and the batch-step "warmuplr" on the device
OPTIM_NAMES = ["adam", "adamw", "sgd", "adadelta", "adagrad", "adamax", "asgd", "lbfgs", "rmsprop", "rprop",
               "radam", "novograd", "sgdw", "adabound", "adamod", "diffgrad", "lamb", "lars", "pid",
               "qhadam", "qhm", "sgdp", "yogi"]
SCHEDULER_NAMES = ["reducelronplateau", "lambdalr", "steplr", "multisteplr", "exponentiallr", "cosineannealinglr",
                   "noamlr", "warmuplr", "piecewiselinearwarmuplr", "warmupsteplr", "warmupreducelronplateau",
                   "cycliclr", "onecyclelr", "cosineannealingwarmrestarts", "cosineannealingwarmuplr"]


def _default_kwargs(cls) -> Dict[str, Any]:
    """get_default_kwargs (espnet2/utils/get_default_kwargs.py): constructor defaults that
    are plain YAML values."""
    out = {}
    try:
        sig = inspect.signature(cls.__init__)
    except (TypeError, ValueError):
        return out
    for name, p in sig.parameters.items():
        if name in ("self",) or p.kind in (p.VAR_POSITIONAL, p.VAR_KEYWORD) or p.default is p.empty:
            continue
        v = p.default
        if isinstance(v, tuple):
            v = list(v)
        if v is None or isinstance(v, (bool, int, float, str, list, dict)):
            out[name] = copy.deepcopy(v)
    return out


def _adam_defaults():
    return dict(lr=0.001, betas=[0.9, 0.999], eps=1.0e-08, weight_decay=0, amsgrad=False)


def _warmuplr_defaults():
    return dict(warmup_steps=25000)


class AbsTask:
    num_optimizers: int = 1
    trainer = Trainer
    class_choices_list: List = []

    # ------------------------------------------------------------------ task hooks
    @classmethod
    def add_task_arguments(cls, parser: argparse.ArgumentParser):
        raise NotImplementedError

    @classmethod
    def build_collate_fn(cls, args, train: bool):
        raise NotImplementedError

    @classmethod
    def build_preprocess_fn(cls, args, train: bool):
        raise NotImplementedError

    @classmethod
    def required_data_names(cls, train: bool = True, inference: bool = False) -> Tuple[str, ...]:
        raise NotImplementedError

    @classmethod
    def optional_data_names(cls, train: bool = True, inference: bool = False) -> Tuple[str, ...]:
        raise NotImplementedError

    @classmethod
    def build_model(cls, args):
        raise NotImplementedError

    # ------------------------------------------------------------------ parser
    @classmethod
    def get_parser(cls) -> ArgumentParser:
        """abs_task.py:261-870 (option names, types, defaults, choices)."""

        class ArgumentDefaultsRawTextHelpFormatter(argparse.RawTextHelpFormatter,
                                                   argparse.ArgumentDefaultsHelpFormatter):
            pass

        parser = ArgumentParser(description="base parser", formatter_class=ArgumentDefaultsRawTextHelpFormatter)
        # "required" is kept in the namespace and checked after --print_config (abs_task.py:267-272)
        parser.set_defaults(required=["output_dir"])
        g = parser.add_argument_group("Common configuration")
        g.add_argument("--print_config", action="store_true", help="Print the config file and exit")
        g.add_argument("--log_level", type=lambda x: x.upper(), default="INFO",
                       choices=("ERROR", "WARNING", "INFO", "DEBUG", "NOTSET"), help="The verbose level of logging")
        g.add_argument("--dry_run", type=str2bool, default=False, help="Perform process without training")
        g.add_argument("--iterator_type", type=str, choices=["sequence", "chunk", "task", "none"], default="sequence",
                       help="Specify iterator type")
        g.add_argument("--output_dir", type=str_or_none, default=None)
        g.add_argument("--ngpu", type=int, default=0, help="The number of gpus. 0 indicates CPU mode")
        g.add_argument("--seed", type=int, default=0, help="Random seed")
        g.add_argument("--num_workers", type=int, default=1, help="The number of workers used for DataLoader")
        g.add_argument("--num_att_plot", type=int, default=3,
                       help="The number images to plot the outputs from attention.")
        g = parser.add_argument_group("distributed training related")
        g.add_argument("--dist_backend", default="nccl", type=str, help="distributed backend")
        g.add_argument("--dist_init_method", type=str, default="env://", help="if init_method='env://'")
        g.add_argument("--dist_world_size", default=None, type=int_or_none, help="number of nodes")
        g.add_argument("--dist_rank", type=int_or_none, default=None, help="node rank")
        g.add_argument("--local_rank", type=int_or_none, default=None, help="local rank")
        g.add_argument("--dist_master_addr", default=None, type=str_or_none, help="master address")
        g.add_argument("--dist_master_port", default=None, type=int_or_none, help="master port")
        g.add_argument("--dist_launcher", default=None, type=str_or_none, choices=["slurm", "mpi", None],
                       help="launcher type")
        g.add_argument("--multiprocessing_distributed", default=False, type=str2bool,
                       help="Use multi-processing distributed training")
        g.add_argument("--unused_parameters", type=str2bool, default=False,
                       help="find_unused_parameters of DistributedDataParallel")
        g.add_argument("--sharded_ddp", default=False, type=str2bool, help="fairscale ShardedDDP")
        g = parser.add_argument_group("cudnn mode related")
        g.add_argument("--cudnn_enabled", type=str2bool, default=torch.backends.cudnn.enabled)
        g.add_argument("--cudnn_benchmark", type=str2bool, default=torch.backends.cudnn.benchmark)
        g.add_argument("--cudnn_deterministic", type=str2bool, default=True)
        g = parser.add_argument_group("collect stats mode related")
        g.add_argument("--collect_stats", type=str2bool, default=False)
        g.add_argument("--write_collected_feats", type=str2bool, default=False)
        g = parser.add_argument_group("Trainer related")
        g.add_argument("--max_epoch", type=int, default=40)
        g.add_argument("--patience", type=int_or_none, default=None)
        g.add_argument("--val_scheduler_criterion", type=str, nargs=2, default=("valid", "loss"))
        g.add_argument("--early_stopping_criterion", type=str, nargs=3, default=("valid", "loss", "min"))
        g.add_argument("--best_model_criterion", type=str2triple_str, nargs="+",
                       default=[("train", "loss", "min"), ("valid", "loss", "min"), ("train", "acc", "max"),
                                ("valid", "acc", "max")])
        g.add_argument("--keep_nbest_models", type=int, nargs="+", default=[10])
        g.add_argument("--nbest_averaging_interval", type=int, default=0)
        g.add_argument("--grad_clip", type=float, default=5.0, help="Gradient norm threshold to clip")
        g.add_argument("--grad_clip_type", type=float, default=2.0, help="The type of the used p-norm")
        g.add_argument("--grad_noise", type=str2bool, default=False)
        g.add_argument("--accum_grad", type=int, default=1)
        g.add_argument("--no_forward_run", type=str2bool, default=False)
        g.add_argument("--resume", type=str2bool, default=False)
        g.add_argument("--train_dtype", default="float32", choices=["float16", "float32", "float64"])
        g.add_argument("--use_amp", type=str2bool, default=False, help="Enable Automatic Mixed Precision")
        g.add_argument("--log_interval", type=int_or_none, default=None)
        g.add_argument("--use_matplotlib", type=str2bool, default=True)
        g.add_argument("--use_tensorboard", type=str2bool, default=True)
        g.add_argument("--create_graph_in_tensorboard", type=str2bool, default=False)
        g.add_argument("--use_wandb", type=str2bool, default=False)
        g.add_argument("--wandb_project", type=str, default=None)
        g.add_argument("--wandb_id", type=str, default=None)
        g.add_argument("--wandb_entity", type=str, default=None)
        g.add_argument("--wandb_name", type=str, default=None)
        g.add_argument("--wandb_model_log_interval", type=int, default=-1)
        g.add_argument("--detect_anomaly", type=str2bool, default=False)
        g = parser.add_argument_group("Pretraining model related")
        g.add_argument("--pretrain_path", help="This option is obsoleted")
        g.add_argument("--init_param", type=str, default=[], nargs="*")
        g.add_argument("--ignore_init_mismatch", type=str2bool, default=False)
        g.add_argument("--freeze_param", type=str, default=[], nargs="*")
        g = parser.add_argument_group("BatchSampler related")
        g.add_argument("--num_iters_per_epoch", type=int_or_none, default=None)
        g.add_argument("--batch_size", type=int, default=20)
        g.add_argument("--valid_batch_size", type=int_or_none, default=None)
        g.add_argument("--batch_bins", type=int, default=1000000)
        g.add_argument("--valid_batch_bins", type=int_or_none, default=None)
        g.add_argument("--train_shape_file", type=str, action="append", default=[])
        g.add_argument("--valid_shape_file", type=str, action="append", default=[])
        g = parser.add_argument_group("Sequence iterator related")
        g.add_argument("--batch_type", type=str, default="folded", choices=list(BATCH_TYPES))
        g.add_argument("--valid_batch_type", type=str_or_none, default=None, choices=list(BATCH_TYPES) + [None])
        g.add_argument("--fold_length", type=int, action="append", default=[])
        g.add_argument("--sort_in_batch", type=str, default="descending", choices=["descending", "ascending"])
        g.add_argument("--sort_batch", type=str, default="descending", choices=["descending", "ascending"])
        g.add_argument("--multiple_iterator", type=str2bool, default=False)
        g = parser.add_argument_group("Chunk iterator related")
        g.add_argument("--chunk_length", type=str_or_int, default=500)
        g.add_argument("--chunk_shift_ratio", type=float, default=0.5)
        g.add_argument("--num_cache_chunks", type=int, default=1024)
        g = parser.add_argument_group("Dataset related")
        g.add_argument("--train_data_path_and_name_and_type", type=str2triple_str, action="append", default=[])
        g.add_argument("--valid_data_path_and_name_and_type", type=str2triple_str, action="append", default=[])
        g.add_argument("--allow_variable_data_keys", type=str2bool, default=False)
        g.add_argument("--max_cache_size", type=parse_size, default=0.0)
        g.add_argument("--max_cache_fd", type=int, default=32)
        g.add_argument("--valid_max_cache_size", type=humanfriendly_parse_size_or_none, default=None)
        g = parser.add_argument_group("Optimizer related")
        g.add_argument("--exclude_weight_decay", type=str2bool, default=False)
        g.add_argument("--exclude_weight_decay_conf", action=NestedDictAction, default=dict())
        for i in range(1, cls.num_optimizers + 1):
            suf = "" if i == 1 else str(i)
            g.add_argument(f"--optim{suf}", type=lambda x: x.lower(), default="adadelta", choices=OPTIM_NAMES)
            g.add_argument(f"--optim{suf}_conf", action=NestedDictAction, default=dict())
            g.add_argument(f"--scheduler{suf}", type=lambda x: str_or_none(x.lower()), default=None,
                           choices=SCHEDULER_NAMES + [None])
            g.add_argument(f"--scheduler{suf}_conf", action=NestedDictAction, default=dict())
        cls.trainer.add_arguments(parser)
        cls.add_task_arguments(parser)
        return parser

    # ------------------------------------------------------------------ config printing
    @classmethod
    def exclude_opts(cls) -> Tuple[str, ...]:
        return "required", "print_config", "config", "ngpu"

    @classmethod
    def get_default_config(cls) -> Dict[str, Any]:
        """abs_task.py:935-985: the defaults, with every class's constructor defaults filled
        into its *_conf."""
        args, _ = cls.get_parser().parse_known_args([])
        config = vars(args)
        for k in cls.exclude_opts():
            config.pop(k, None)
        for i in range(1, cls.num_optimizers + 1):
            suf = "" if i == 1 else str(i)
            if config[f"optim{suf}"] == "adam":
                config[f"optim{suf}_conf"] = dict(_adam_defaults(), **config[f"optim{suf}_conf"])
            if config[f"scheduler{suf}"] == "warmuplr":
                config[f"scheduler{suf}_conf"] = dict(_warmuplr_defaults(), **config[f"scheduler{suf}_conf"])
        for cc in cls.class_choices_list:
            name = config.get(cc.name)
            # a default the build does not register (e.g. encoder "rnn") keeps its given conf
            if name is not None and str(name).lower() in cc.classes:
                conf = _default_kwargs(cc.get_class(name))
                conf.update(config[f"{cc.name}_conf"])
                config[f"{cc.name}_conf"] = conf
        return config

    @classmethod
    def print_config(cls, file=None) -> None:
        file = sys.stdout if file is None else file
        file.write(yaml.safe_dump(_yaml_friendly(cls.get_default_config()), indent=4, sort_keys=False))

    @classmethod
    def check_required_command_args(cls, args):
        for k in vars(args):
            if "-" in k:
                raise RuntimeError(f'Use "_" instead of "-": parser.get_parser("{k}")')
        missing = ", ".join(f"--{a}" for a in args.required if getattr(args, a, None) is None)
        if missing:
            cls.get_parser().print_help(file=sys.stderr)
            print(f"\n{Path(sys.argv[0]).name}: error: the following arguments are required: {missing}",
                  file=sys.stderr)
            sys.exit(2)

    @classmethod
    def check_task_requirements(cls, dataset, allow_variable_data_keys: bool, train: bool, inference: bool = False):
        mes = (f'If you intend to use an additional input, modify "{cls.__name__}.required_data_names()" or '
               f'"{cls.__name__}.optional_data_names()". Otherwise you need to set --allow_variable_data_keys true ')
        for k in cls.required_data_names(train, inference):
            if not dataset.has_name(k):
                raise RuntimeError(f'"{cls.required_data_names(train, inference)}" are required for {cls.__name__}. '
                                   f'but "{dataset.names()}" are input.\n{mes}')
        if not allow_variable_data_keys:
            task_keys = cls.required_data_names(train, inference) + cls.optional_data_names(train, inference)
            for k in dataset.names():
                if k not in task_keys:
                    raise RuntimeError(f"The data-name must be one of {task_keys} for {cls.__name__}: "
                                       f'"{k}" is not allowed.\n{mes}')

    # ------------------------------------------------------------------ optimizers
    @classmethod
    def build_optimizers(cls, args, model) -> List:
        """abs_task.py:872-903 for optim "adam" over the parameter arena (frozen parameters
        and exclude_weight_decay are not supported by the arena Adam)."""
        from ..optim.adam import ArenaAdam
        if args.optim != "adam":
            raise NotImplementedError(f"--optim {args.optim}: the MI355X build runs the arena Adam "
                                      "(--optim adam, the conformer recipes' optimizer)")
        if args.exclude_weight_decay:
            raise NotImplementedError("--exclude_weight_decay true")
        conf = dict(args.optim_conf)
        if "betas" in conf:
            conf["betas"] = tuple(conf["betas"])
        return [ArenaAdam(model, **conf)]

    @classmethod
    def build_schedulers(cls, args, optimizers) -> List:
        from ..schedulers.warmup_lr import WarmupLR
        out = []
        for i, opt in enumerate(optimizers, 1):
            suf = "" if i == 1 else str(i)
            name = getattr(args, f"scheduler{suf}")
            conf = getattr(args, f"scheduler{suf}_conf")
            if name is None:
                out.append(None)
            elif name == "warmuplr":
                out.append(WarmupLR(opt, **conf))
            else:
                raise NotImplementedError(f"--scheduler {name}: the build evaluates warmuplr on the device")
        return out

    # ------------------------------------------------------------------ iterators
    @classmethod
    def build_iter_factory(cls, args, distributed_option: DistributedOption, mode: str):
        """abs_task.py:1362-1575 (iterator_type sequence)."""
        if args.iterator_type != "sequence":
            raise NotImplementedError(f"--iterator_type {args.iterator_type}")
        if args.multiple_iterator:
            raise NotImplementedError("--multiple_iterator true")
        train = mode == "train"
        if train:
            data = args.train_data_path_and_name_and_type
            shape_files = args.train_shape_file
            batch_type, batch_size, batch_bins = args.batch_type, args.batch_size, args.batch_bins
            num_iters = args.num_iters_per_epoch
        elif mode == "valid":
            data = args.valid_data_path_and_name_and_type
            shape_files = args.valid_shape_file
            batch_type = args.batch_type if args.valid_batch_type is None else args.valid_batch_type
            batch_size = args.batch_size if args.valid_batch_size is None else args.valid_batch_size
            batch_bins = args.batch_bins if args.valid_batch_bins is None else args.valid_batch_bins
            num_iters = None
        else:
            raise NotImplementedError(f"mode={mode}")
        dataset = ESPnetDataset(data, float_dtype=args.train_dtype, preprocess=cls.build_preprocess_fn(args, train))
        cls.check_task_requirements(dataset, args.allow_variable_data_keys, train=train)
        cat = Path(Path(data[0][0]).parent, "utt2category")
        sampler = build_batch_sampler(type=batch_type, shape_files=shape_files, fold_lengths=args.fold_length,
                                      batch_size=batch_size, batch_bins=batch_bins, sort_in_batch=args.sort_in_batch,
                                      sort_batch=args.sort_batch, drop_last=False,
                                      min_batch_size=torch.distributed.get_world_size()
                                      if distributed_option.distributed else 1,
                                      utt2category_file=str(cat) if cat.exists() else None)
        batches = list(sampler)
        bs = [len(b) for b in batches]
        logging.info(f"[{mode}] dataset:\n{dataset}")
        logging.info(f"[{mode}] Batch sampler: {sampler}")
        logging.info(f"[{mode}] mini-batch sizes summary: N-batch={len(bs)}, mean={np.mean(bs):.1f}, "
                     f"min={np.min(bs)}, max={np.max(bs)}")
        if distributed_option.distributed:
            world = torch.distributed.get_world_size()
            rank = torch.distributed.get_rank()
            for b in batches:
                if len(b) < world:
                    raise RuntimeError(f"The batch-size must be equal or more than world_size: {len(b)} < {world}")
            batches = [b[rank::world] for b in batches]  # abs_task.py:1566-1575
        return SequenceIterFactory(dataset=dataset, batches=batches, seed=args.seed, num_iters_per_epoch=num_iters,
                                   shuffle=train, num_workers=args.num_workers,
                                   collate_fn=cls.build_collate_fn(args, train), pin_memory=args.ngpu > 0)

    # ------------------------------------------------------------------ entry points
    @classmethod
    def normalize_args(cls, args: argparse.Namespace) -> argparse.Namespace:
        """A YAML config sets values without type conversion (config_argparse.py:40-45), so
        recipe keys like `patience: none` / `init: none` arrive as the string "none"; map
        those to None where the option's default is None (what the command-line type
        str_or_none / int_or_none would have produced)."""
        defaults = vars(cls.get_parser().parse_known_args([])[0])
        for k, v in vars(args).items():
            if isinstance(v, str) and v.strip().lower() in ("none", "null", "nil") and defaults.get(k, 0) is None:
                setattr(args, k, None)
        return args

    @classmethod
    def main(cls, args: argparse.Namespace = None, cmd: Sequence[str] = None):
        if args is None:
            args = cls.get_parser().parse_args(cmd)
        cls.normalize_args(args)
        if args.pretrain_path is not None:
            raise RuntimeError("--pretrain_path is deprecated. Use --init_param")
        if args.print_config:
            cls.print_config()
            sys.exit(0)
        cls.check_required_command_args(args)
        resolve_distributed_mode(args)
        if not args.distributed or not args.multiprocessing_distributed:
            cls.main_worker(args)
            return
        # one spawned worker per GPU of this node (abs_task.py:1041-1094)
        assert args.ngpu > 1, args.ngpu
        args.dist_master_addr = "127.0.0.1"
        args.dist_rank = 0
        if args.dist_init_method == "env://" and args.dist_master_port is None and "MASTER_PORT" not in os.environ:
            args.dist_master_port = free_port()
        args.dist_world_size = args.ngpu
        ctx = torch.multiprocessing.get_context("spawn")
        procs = []
        for i in range(args.ngpu):
            local = argparse.Namespace(**vars(args))
            local.local_rank = i
            local.dist_rank = i
            local.ngpu = 1
            p = ctx.Process(target=cls.main_worker, args=(local,), daemon=False)
            p.start()
            procs.append(p)
        failed = []
        for p in procs:
            p.join()
            if p.exitcode != 0:
                failed.append(p.exitcode)
        if failed:
            raise RuntimeError(f"worker(s) exited with {failed}")

    @classmethod
    def _unsupported(cls, args):
        bad = []
        for key, default in (("sharded_ddp", False), ("grad_noise", False), ("use_wandb", False),
                             ("collect_stats", False), ("detect_anomaly", False), ("create_graph_in_tensorboard", False),
                             ("freeze_param", [])):
            if getattr(args, key, default) not in (default, None):
                bad.append(f"--{key} {getattr(args, key)}")
        if args.train_dtype != "float32":
            bad.append(f"--train_dtype {args.train_dtype}")
        if args.grad_clip_type != 2.0:
            bad.append(f"--grad_clip_type {args.grad_clip_type}")
        if args.ngpu < 1:
            bad.append("--ngpu 0 (the build runs on the GPU only; the CPU path is the reference's)")
        if bad:
            raise NotImplementedError("not supported by the MI355X build: " + ", ".join(bad))

    @classmethod
    def main_worker(cls, args: argparse.Namespace):
        dopt = DistributedOption(**{f.name: getattr(args, f.name) for f in DistributedOption.__dataclass_fields__.values()
                                    if hasattr(args, f.name)})
        dopt.init_options()
        rank0 = not dopt.distributed or dopt.dist_rank == 0
        logging.basicConfig(level=args.log_level if rank0 else "ERROR",
                            format=f"[{os.uname()[1].split('.')[0]}"
                                   + (f":{dopt.dist_rank}/{dopt.dist_world_size}" if dopt.distributed else "")
                                   + "] %(asctime)s (%(module)s:%(lineno)d) %(levelname)s: %(message)s")
        cls._unsupported(args)
        dopt.init_torch_distributed()
        _set_all_random_seed(args.seed)
        model = cls.build_model(args=args)
        device = torch.device("cuda", dopt.device_index() if dopt.local_rank is not None
                              else torch.cuda.current_device())
        torch.cuda.set_device(device)
        for p in args.init_param:
            _load_pretrained(model, p, args.ignore_init_mismatch)
        model.prepare(device, amp=bool(args.use_amp), seed=args.seed)
        optimizers = cls.build_optimizers(args, model)
        schedulers = cls.build_schedulers(args, optimizers)
        output_dir = Path(args.output_dir)
        if rank0:
            output_dir.mkdir(parents=True, exist_ok=True)
            with (output_dir / "config.yaml").open("w", encoding="utf-8") as f:
                yaml.safe_dump(_yaml_friendly(vars(args)), f, indent=4, sort_keys=False)
        if args.dry_run:
            return
        train_iter = cls.build_iter_factory(args, dopt, "train")
        valid_iter = cls.build_iter_factory(args, dopt, "valid")
        options = cls.trainer.build_options(args)
        cls.trainer.run(model=model, optimizers=optimizers, schedulers=schedulers, train_iter_factory=train_iter,
                        valid_iter_factory=valid_iter, plot_attention_iter_factory=None, trainer_options=options,
                        distributed_option=dopt)
        if dopt.distributed:
            torch.distributed.destroy_process_group()


def _set_all_random_seed(seed: int):
    """espnet2/torch_utils/set_all_random_seed.py."""
    import random
    random.seed(seed)
    np.random.seed(seed)
    torch.random.manual_seed(seed)


def _load_pretrained(model, init_param: str, ignore_init_mismatch: bool):
    """load_pretrained_model (espnet2/torch_utils/load_pretrained_model.py) for
    "<file>[:<src_key>[:<dst_key>[:<exclude_keys>]]]"; weights_only loading."""
    sps = init_param.split(":", 4)
    path = sps[0]
    src_key = sps[1] if len(sps) > 1 and sps[1] else None
    dst_key = sps[2] if len(sps) > 2 and sps[2] else None
    excludes = sps[3].split(",") if len(sps) > 3 and sps[3] else []
    obj = model if dst_key is None else model.get_submodule(dst_key)
    src = torch.load(path, map_location="cpu", weights_only=True)
    if src_key is not None:
        src = {k[len(src_key) + 1:]: v for k, v in src.items() if k.startswith(src_key + ".")}
    src = {k: v for k, v in src.items() if not any(k.startswith(e) for e in excludes)}
    dst = obj.state_dict()
    if ignore_init_mismatch:
        src = {k: v for k, v in src.items() if k in dst and dst[k].shape == v.shape}
    dst.update(src)
    obj.load_state_dict(dst)


def _yaml_friendly(x):
    if isinstance(x, dict):
        return {k: _yaml_friendly(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_yaml_friendly(v) for v in x]
    if isinstance(x, Path):
        return str(x)
    if x is None or isinstance(x, (bool, int, float, str)):
        return x
    return str(x)
