"""Disassemble one kernel of a built object and list its vmcnt waits, barriers, LDS-DMA and
scratch accesses with their line numbers (pipelining checks), plus an instruction histogram.

    python scripts/isa_scan.py relattn attn_bwdq2_kernelILb1 [--hist]
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
obj = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "espnet-1_amd", "build", "obj",
                   sys.argv[1] + ".hip.o")
pat = sys.argv[2]
with tempfile.TemporaryDirectory() as d:
    fat, co = os.path.join(d, "fat.bin"), os.path.join(d, "k.co")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj, os.path.join(d, "x.o")],
                   check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    s = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], capture_output=True,
                       text=True).stdout.split("\n")
start = [i for i, l in enumerate(s) if re.match(r"^[0-9a-f]+ <.*" + pat, l)][0]
end = next((i for i, l in enumerate(s) if i > start and re.match(r"^[0-9a-f]+ <", l)), len(s))
body = s[start:end]
hist = {}
for i, l in enumerate(body):
    t = l.strip().split()
    if t:
        hist[t[0]] = hist.get(t[0], 0) + 1
    if any(k in l for k in ("vmcnt", "s_barrier", "global_load_lds", "scratch_")) or re.search(r"s_cbranch\S* 6\d{4}", l):
        print(i, l.strip()[:96])
if "--hist" in sys.argv:
    for k, v in sorted(hist.items(), key=lambda kv: -kv[1])[:40]:
        print(f"{v:6d} {k}")
