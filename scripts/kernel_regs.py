"""VGPR / spill / LDS per kernel of a built object (gfx950 code object inside the host .o).

    python scripts/kernel_regs.py relattn [name-substring ...]
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
obj = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "espnet-1_amd", "build", "obj",
                   sys.argv[1] + ".hip.o")
pats = sys.argv[2:]
with tempfile.TemporaryDirectory() as d:
    fat, co = os.path.join(d, "fat.bin"), os.path.join(d, "k.co")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj, os.path.join(d, "x.o")],
                   check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
for blk in notes.split("- .agpr_count")[1:]:
    name = re.search(r"\.name:\s+(\S+)", blk).group(1)
    if pats and not any(p in name for p in pats):
        continue
    g = lambda k: (re.search(r"\." + k + r":\s+(\S+)", blk) or [None, None])[1]  # noqa: E731
    print(f"{name[:90]:90s} vgpr {g('vgpr_count'):>4s} spill {g('vgpr_spill_count'):>3s} "
          f"priv {g('private_segment_fixed_size'):>4s} lds {g('group_segment_fixed_size'):>6s}")
