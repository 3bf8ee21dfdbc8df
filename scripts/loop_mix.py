"""Instruction mix of the hottest loop(s) of a kernel in a built object: for each backward
branch (loop), the instructions between its target and the branch, by class.

    python scripts/loop_mix.py relattn attn_bwdkv_kernelILb1
"""
import collections
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
    asm = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], capture_output=True,
                         text=True).stdout
for f in re.split(r"\n(?=[0-9a-f]+ <[^>]+>:)", asm):
    m = re.match(r"([0-9a-f]+) <([^>]+)>:", f)
    if not m or pat not in m.group(2):
        continue
    ins = []
    for line in f.split("\n")[1:]:
        mm = re.match(r"\s*([a-z_0-9]+)\s*(.*?)\s*//\s*([0-9A-F]+):(.*)", line)
        if mm:
            ins.append((int(mm.group(3), 16), mm.group(1), mm.group(2) + mm.group(4)))
    addr = {a: k for k, (a, _, _) in enumerate(ins)}
    print(m.group(2)[:80], len(ins), "instructions")
    for k, (a, op, args) in enumerate(ins):
        if op.startswith("s_cbranch") or op == "s_branch":
            t = re.search(r"<[^+]+\+0x([0-9a-f]+)>", args)
            if not t:
                continue
            tgt = int(m.group(1), 16) + int(t.group(1), 16)
            if tgt < a and tgt in addr and k - addr[tgt] > 50:
                body = ins[addr[tgt]:k + 1]
                c = collections.Counter()
                for _, o, _ in body:
                    c["mfma" if "mfma" in o else o.split("_")[0] + "_" + o.split("_")[1] if o.startswith(("ds_", "global_", "buffer_", "scratch_")) else ("valu" if o.startswith("v_") else "salu" if o.startswith("s_") else o)] += 1
                print(f"  loop {tgt:x}..{a:x}: {len(body)} instr", dict(c.most_common()))
    if len(sys.argv) > 3:  # dump the largest loop's VALU histogram / listing
        best = None
        for k, (a, op, args) in enumerate(ins):
            if op.startswith("s_cbranch") or op == "s_branch":
                t = re.search(r"<[^+]+\+0x([0-9a-f]+)>", args)
                if t:
                    tgt = int(m.group(1), 16) + int(t.group(1), 16)
                    if tgt < a and tgt in addr and (best is None or k - addr[tgt] > best[1] - best[0]):
                        best = (addr[tgt], k)
        body = ins[best[0]:best[1] + 1]
        if sys.argv[3] == "hist":
            print(collections.Counter(o for _, o, _ in body if o.startswith("v_")).most_common(40))
        else:
            for _, o, a_ in body:
                print(o, a_.split("//")[0][:70])
