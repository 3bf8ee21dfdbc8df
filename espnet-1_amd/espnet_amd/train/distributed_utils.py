"""DistributedOption / resolve_distributed_mode — espnet2/train/distributed_utils.py:9-166
for one node: RANK / WORLD_SIZE / LOCAL_RANK / MASTER_* from the arguments or the
environment (torchrun), one process per GPU.  backend "nccl" is RCCL on ROCm (over xGMI);
HSA_ENABLE_IPC_MODE_LEGACY=0 is kept in the environment (the dmabuf IPC the MI355X host
driver supports).  Besides the device group, a gloo group over the same ranks carries the
host-side control flags (the per-step iterator_stop of trainer.py:507-518), so they never
synchronise a GPU stream.  The SLURM / MPI launchers are not supported (cluster plumbing
outside the training step)."""
from __future__ import annotations

import dataclasses
import os
import socket
from typing import Optional

import torch
import torch.distributed as dist


def _env_int(name) -> Optional[int]:
    v = os.environ.get(name)
    return None if v is None else int(v)


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@dataclasses.dataclass
class DistributedOption:
    distributed: bool = False
    dist_backend: str = "nccl"
    dist_init_method: str = "env://"
    dist_world_size: Optional[int] = None
    dist_rank: Optional[int] = None
    local_rank: Optional[int] = None
    ngpu: int = 0
    dist_master_addr: Optional[str] = None
    dist_master_port: Optional[int] = None
    dist_launcher: Optional[str] = None
    multiprocessing_distributed: bool = True

    control_group = None  # gloo group for host-side flags

    def init_options(self):
        if not self.distributed:
            return
        if self.dist_launcher is not None:
            raise NotImplementedError(f"dist_launcher={self.dist_launcher}: use torchrun or "
                                      "--multiprocessing_distributed true on one node")
        if self.dist_init_method == "env://":
            if (self.dist_master_addr or os.environ.get("MASTER_ADDR")) is None:
                raise RuntimeError("--dist_master_addr or MASTER_ADDR must be set if --dist_init_method == 'env://'")
            if (self.dist_master_port or _env_int("MASTER_PORT")) is None:
                raise RuntimeError("--dist_master_port or MASTER_PORT must be set if --dist_init_port == 'env://'")
        self.dist_rank = self.dist_rank if self.dist_rank is not None else _env_int("RANK")
        self.dist_world_size = self.dist_world_size if self.dist_world_size is not None else _env_int("WORLD_SIZE")
        self.local_rank = self.local_rank if self.local_rank is not None else _env_int("LOCAL_RANK")
        if self.local_rank is not None and self.ngpu > 1:
            raise RuntimeError(f"Assuming 1GPU in this case: ngpu={self.ngpu}")
        if self.dist_rank is not None and self.dist_world_size is not None and self.dist_rank >= self.dist_world_size:
            raise RuntimeError(f"RANK >= WORLD_SIZE: {self.dist_rank} >= {self.dist_world_size}")
        if self.dist_init_method == "env://":
            addr = self.dist_master_addr or os.environ.get("MASTER_ADDR")
            port = self.dist_master_port or _env_int("MASTER_PORT")
            self.dist_master_addr, self.dist_master_port = addr, port
            self.dist_init_method = f"tcp://{addr}:{port}"

    def device_index(self) -> Optional[int]:
        """This worker's GPU.  RCCL needs one GPU per rank (local_rank); with a host transport
        (gloo) ranks beyond the node's GPU count share them round-robin, which is how the
        multi-worker entry point is rehearsed on a one-GPU box (bench.py does the same)."""
        if self.local_rank is None:
            return None
        if self.dist_backend != "nccl":
            return self.local_rank % max(1, torch.cuda.device_count())
        return self.local_rank

    def init_torch_distributed(self):
        if not self.distributed:
            return
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if self.dist_backend == "nccl":
            from .graph import prepare_nccl_env
            prepare_nccl_env()
        kwargs = {}
        if self.ngpu > 0 and self.local_rank is not None:
            torch.cuda.set_device(self.device_index())
            if self.dist_backend == "nccl":
                kwargs["device_id"] = torch.device("cuda", self.device_index())
        dist.init_process_group(backend=self.dist_backend, init_method=self.dist_init_method,
                                world_size=self.dist_world_size, rank=self.dist_rank, **kwargs)
        self.control_group = dist.new_group(backend="gloo") if self.dist_backend != "gloo" else None


def resolve_distributed_mode(args):
    """distributed_utils.py:112-166 for a single node (launchers none / torchrun)."""
    if args.multiprocessing_distributed:
        args.distributed = args.ngpu > 1
        if args.ngpu <= 1:
            args.multiprocessing_distributed = False
        if args.ngpu == 1:
            args.local_rank = 0
    else:
        ws = args.dist_world_size if args.dist_world_size is not None else _env_int("WORLD_SIZE")
        args.distributed = ws is not None and ws > 1
        if args.distributed and args.ngpu > 0 and (args.local_rank if args.local_rank is not None
                                                   else _env_int("LOCAL_RANK")) is None:
            raise RuntimeError("--local_rank or LOCAL_RANK must be set if --multiprocessing_distributed == false")
        if args.distributed and (args.dist_rank if args.dist_rank is not None else _env_int("RANK")) is None:
            raise RuntimeError("--dist_rank or RANK must be set if --multiprocessing_distributed == false")
