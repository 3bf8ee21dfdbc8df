"""Build an experiment variant of libespnet_amd.so: the named csrc files recompiled with extra
preprocessor definitions, everything else from the working tree's objects, linked as
espnet_amd/lib/libespnet_amd_<tag>.so (load it with EA_LIB_NAME=libespnet_amd_<tag>.so).

    python scripts/build_def.py TAG "-DFOO=1 -DBAR=2" csrc/relattn.hip [...]
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "espnet-1_amd")
sys.path.insert(0, PKG)
import build as B  # noqa: E402


def main():
    tag, defs, files = sys.argv[1], sys.argv[2].split(), sys.argv[3:]
    B.build(verbose=False)
    objs = []
    for s in sorted(os.listdir(B.CSRC)):
        if not s.endswith(".hip"):
            continue
        if f"csrc/{s}" in files:
            obj = os.path.join(B.OBJ, f"{s}.{tag}.o")
            subprocess.run([B.HIPCC, *B.CFLAGS, *defs, "-c", os.path.join(B.CSRC, s), "-o", obj], check=True)
            objs.append(obj)
        else:
            objs.append(os.path.join(B.OBJ, s + ".o"))
    out = os.path.join(PKG, "espnet_amd", "lib", f"libespnet_amd_{tag}.so")
    subprocess.run([B.HIPCC, "-shared", f"--offload-arch={B.ARCH}", "-o", out, *objs], check=True)
    print("built", out)


if __name__ == "__main__":
    main()
