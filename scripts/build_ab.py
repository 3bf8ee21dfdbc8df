"""Build an A/B variant of libespnet_amd.so: the named csrc files taken from a git revision,
everything else from the working tree, linked as espnet_amd/lib/libespnet_amd_<tag>.so (load it
with EA_LIB_NAME=libespnet_amd_<tag>.so).

    python scripts/build_ab.py TAG REV csrc/relattn.hip [csrc/gemm_kern.h ...]
"""
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "espnet-1_amd")
sys.path.insert(0, PKG)
import build as B  # noqa: E402


def main():
    tag, rev, files = sys.argv[1], sys.argv[2], sys.argv[3:]
    B.build(verbose=False)
    with tempfile.TemporaryDirectory() as d:
        csrc = os.path.join(d, "pkg", "csrc")  # common.h includes ../../include/espnet_amd.h
        shutil.copytree(B.CSRC, csrc)
        shutil.copytree(B.INCLUDE, os.path.join(d, "include"))
        for f in files:
            src = subprocess.run(["git", "show", f"{rev}:espnet-1_amd/{f}"], cwd=ROOT, capture_output=True,
                                 text=True, check=True).stdout
            open(os.path.join(d, "pkg", f), "w").write(src)
        hdr_changed = any(f.endswith(".h") for f in files)
        objs = []
        for s in sorted(os.listdir(csrc)):
            if not s.endswith(".hip"):
                continue
            own = os.path.join(B.OBJ, s + ".o")
            if hdr_changed or f"csrc/{s}" in files:
                obj = os.path.join(d, s + ".o")
                subprocess.run([B.HIPCC, *B.CFLAGS, "-c", os.path.join(csrc, s), "-o", obj], check=True)
                objs.append(obj)
            else:
                objs.append(own)
        out = os.path.join(PKG, "espnet_amd", "lib", f"libespnet_amd_{tag}.so")
        subprocess.run([B.HIPCC, "-shared", f"--offload-arch={B.ARCH}", "-o", out, *objs], check=True)
        print("built", out)


if __name__ == "__main__":
    main()
