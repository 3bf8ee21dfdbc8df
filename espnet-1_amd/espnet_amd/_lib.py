"""ctypes binding of libespnet_amd.so (the C ABI in include/espnet_amd.h).

The argument types are derived from the header's prototypes, so the Python side and the
C ABI cannot drift.  Loading fails loudly when the library is missing: there is no CPU
or PyTorch fallback for any op on the hot path.
"""
from __future__ import annotations

import ctypes
import os
import re

# torch must be loaded BEFORE libespnet_amd.so: the PyTorch-ROCm wheel bundles its own
# libamdhip64.so (soname libamdhip64.so.7).  Loading torch first makes our library's
# libamdhip64.so.7 dependency resolve to that already-loaded runtime, so torch's streams
# and allocations and our kernel launches share ONE HIP runtime in the process.
import torch  # noqa: F401,E402

_PKG = os.path.dirname(os.path.abspath(__file__))
# EA_LIB_NAME selects another in-tree build of the same library (A/B measurements)
LIB_PATH = os.path.join(_PKG, "lib", os.environ.get("EA_LIB_NAME", "libespnet_amd.so"))
HEADER = os.path.join(os.path.dirname(os.path.dirname(_PKG)), "include", "espnet_amd.h")

F32, BF16 = 0, 1
GEMM_PIPE = int(os.environ.get("EA_GEMM_PIPE", "1"))
ACT_NONE, ACT_SWISH, ACT_RELU = 0, 1, 2
EPI_STORE, EPI_ACT, EPI_RESID, EPI_DACT = 0, 1, 2, 3
ERR_BAD_ARG = 1000


class Epilogue(ctypes.Structure):
    _fields_ = [
        ("kind", ctypes.c_int), ("act", ctypes.c_int),
        ("alpha", ctypes.c_float), ("beta", ctypes.c_float), ("post_scale", ctypes.c_float),
        ("rscale", ctypes.c_float), ("drop_p", ctypes.c_float),
        ("seed", ctypes.c_ulonglong),
        ("bias", ctypes.c_void_p),
        ("aux", ctypes.c_void_p), ("aux_dtype", ctypes.c_int), ("ldaux", ctypes.c_long),
        ("resid", ctypes.c_void_p), ("ldr", ctypes.c_long),
    ]


class GroupGemm(ctypes.Structure):
    """ea_group_gemm: one problem of ea_gemm_grouped."""
    _fields_ = [("A", ctypes.c_void_p), ("B", ctypes.c_void_p), ("C", ctypes.c_void_p),
                ("lda", ctypes.c_long), ("ldb", ctypes.c_long), ("ldc", ctypes.c_long),
                ("M", ctypes.c_int), ("N", ctypes.c_int), ("K", ctypes.c_int), ("beta", ctypes.c_float)]


class ColsumProb(ctypes.Structure):
    """ea_colsum_prob: one column-sum problem of ea_colsum_grouped."""
    _fields_ = [("x", ctypes.c_void_p), ("part", ctypes.c_void_p), ("ld", ctypes.c_long),
                ("rows", ctypes.c_int), ("n", ctypes.c_int), ("dtype", ctypes.c_int), ("rpp", ctypes.c_int)]


class ReduceProb(ctypes.Structure):
    """ea_reduce_prob: one ordered partial-sum reduction of ea_reduce_grouped."""
    _fields_ = [("part", ctypes.c_void_p), ("out", ctypes.c_void_p), ("stride", ctypes.c_long),
                ("nparts", ctypes.c_int), ("n", ctypes.c_int), ("accumulate", ctypes.c_int)]


SCHED_CONSTANT, SCHED_WARMUP = 0, 1
CONV_FWD, CONV_DGRAD, CONV_WGRAD = 1, 2, 3


class ConvGeo(ctypes.Structure):
    """ea_conv_geo: phase-split implicit-GEMM geometry of the subsampling conv2."""
    _fields_ = [("mode", ctypes.c_int), ("B", ctypes.c_int), ("T2", ctypes.c_int), ("F2", ctypes.c_int),
                ("C", ctypes.c_int), ("P", ctypes.c_int), ("nI", ctypes.c_int * 2), ("nJ", ctypes.c_int * 2),
                ("a", ctypes.c_int), ("e", ctypes.c_int), ("plane", ctypes.c_long * 4), ("zero", ctypes.c_long)]


class LrSchedule(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int), ("warmup_steps", ctypes.c_float), ("base_lr", ctypes.c_double)]


# ea_opt_state (device memory, 40 B): step i64 | lr bc1 bc2_sqrt coef last_norm f32 | skip i32 |
# next_lr f32 | pad
OPT_STATE_BYTES = 40
OPT_STATE_NEXT_LR = 8  # float index of next_lr


_CTYPES = {
    "int": ctypes.c_int,
    "long": ctypes.c_long,
    "float": ctypes.c_float,
    "double": ctypes.c_double,
    "unsigned long long": ctypes.c_ulonglong,
    "unsigned int": ctypes.c_uint,
}


def _arg_ctype(decl: str):
    decl = decl.strip()
    if "ea_epilogue" in decl and "*" in decl:
        return ctypes.POINTER(Epilogue)
    if "*" in decl:
        return ctypes.c_void_p
    base = re.sub(r"\bconst\b", "", decl).strip()
    base = " ".join(base.split()[:-1])  # drop the parameter name
    if base not in _CTYPES:
        raise TypeError(f"unsupported C type in header: {decl!r}")
    return _CTYPES[base]


def parse_header(path: str = HEADER):
    """-> {name: [ctypes arg types]} for every `int ea_*(...)` prototype."""
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    protos = {}
    for m in re.finditer(r"\bint\s+(ea_\w+)\s*\(([^)]*)\)\s*;", src):
        name, args = m.group(1), m.group(2)
        args = [a for a in (x.strip() for x in args.split(",")) if a and a != "void"]
        protos[name] = [_arg_ctype(a) for a in args]
    return protos


class HipError(RuntimeError):
    pass


class _Lib:
    def __init__(self):
        self._dll = None
        self.protos = parse_header()

    def load(self):
        if self._dll is None:
            if not os.path.exists(LIB_PATH):
                raise HipError(
                    f"{LIB_PATH} not found: build the HIP library first "
                    "(python espnet-1_amd/build.py). There is no CPU fallback.")
            dll = ctypes.CDLL(LIB_PATH)
            for name, argtypes in self.protos.items():
                fn = getattr(dll, name)
                fn.argtypes = argtypes
                fn.restype = ctypes.c_int
            # 256x256 GEMM tiles on the ping-pong kernel (gemm_pipe); EA_GEMM_PIPE=0 for A/B
            dll.ea_gemm_set_pipe(GEMM_PIPE)
            self._dll = dll
        return self._dll

    def __getattr__(self, name):
        if not name.startswith("ea_"):
            raise AttributeError(name)
        fn = getattr(self.load(), name)

        def call(*args):
            rc = fn(*args)
            if rc != 0:
                what = "bad argument/shape/alignment" if rc == ERR_BAD_ARG else f"hipError {rc}"
                raise HipError(f"{name} failed: {what}")
            return rc

        call.__name__ = name
        setattr(self, name, call)
        return call


lib = _Lib()
