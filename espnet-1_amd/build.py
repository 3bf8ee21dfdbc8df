"""Build libespnet_amd.so (all HIP kernels, gfx950) in-tree.

    python espnet-1_amd/build.py [-j N] [--force]

Each csrc/*.hip is compiled to an object with hipcc --offload-arch=gfx950 (in parallel,
skipped when up to date), then linked into espnet_amd/lib/libespnet_amd.so.  The .so is
git-ignored but travels to the GPU box with the gpurun snapshot.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
OBJ = os.path.join(HERE, "build", "obj")
LIB = os.path.join(HERE, "espnet_amd", "lib", "libespnet_amd.so")
ARCH = os.environ.get("ESPNET_AMD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
          "-Wno-pass-failed", f"-I{INCLUDE}"]


def _deps(src):
    return [src] + glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(INCLUDE, "*.h"))


def _stale(out, deps):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps)


def _file_flags(src):
    """Per-file hipcc flags from a `// hipcc-flags: ...` line in the first lines of the source."""
    with open(src) as f:
        for _, line in zip(range(20), f):
            if line.startswith("// hipcc-flags:"):
                return line.split(":", 1)[1].split()
    return []


def _compile(src, force, obj_dir=OBJ, extra=()):
    obj = os.path.join(obj_dir, os.path.basename(src) + ".o")
    if not force and not _stale(obj, _deps(src)):
        return obj, None
    cmd = [HIPCC, *CFLAGS, *_file_flags(src), *extra, "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        return obj, f"{' '.join(cmd)}\n{r.stdout}\n{r.stderr}"
    return obj, None


def build(jobs: int = 8, force: bool = False, verbose: bool = True, tag: str = "", extra=()) -> str:
    """tag / extra: an A/B variant built with extra hipcc flags into its own object directory,
    linked as libespnet_amd_<tag>.so (load it with EA_LIB_NAME)."""
    obj_dir = OBJ + (f"_{tag}" if tag else "")
    lib = LIB if not tag else LIB.replace(".so", f"_{tag}.so")
    os.makedirs(obj_dir, exist_ok=True)
    os.makedirs(os.path.dirname(lib), exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        results = list(ex.map(lambda s: _compile(s, force, obj_dir, extra), srcs))
    errs = [e for _, e in results if e]
    if errs:
        raise RuntimeError("HIP compile failed:\n" + "\n".join(errs))
    objs = [o for o, _ in results]
    if force or _stale(lib, objs):
        cmd = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-o", lib, *objs]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
        if verbose:
            print(f"[espnet_amd] linked {lib} ({len(objs)} objects)")
    return lib


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", type=int, default=min(8, os.cpu_count() or 8))
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--tag", default="", help="A/B variant: libespnet_amd_<tag>.so")
    ap.add_argument("--extra", default="", help="extra hipcc flags for the variant (space separated)")
    a = ap.parse_args()
    try:
        build(a.j, a.force, tag=a.tag, extra=a.extra.split())
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
