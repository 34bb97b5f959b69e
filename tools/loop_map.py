#!/usr/bin/env python3
"""Static loop map of one kernel in a hipcc object: every backward branch
(s_cbranch_* / s_branch to a lower address) is a loop; for each, its size and
its vector-memory instructions by kind (scratch / global / buffer, load /
store, width).  Used to find the loops whose private-segment traffic is
spills or per-sample accesses.

  python tools/loop_map.py build/obj/libmelpe_amd/k_ana.o k_enc_anaILi1 [min_mem]
"""
import collections
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def disasm(obj):
    with tempfile.TemporaryDirectory() as tmp:
        fat, elf = os.path.join(tmp, "fat.bin"), os.path.join(tmp, "dev.elf")
        subprocess.run(["objcopy", "--dump-section", ".hip_fatbin=" + fat, obj], check=True)
        subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                        "--input=" + fat, "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                        "--output=" + elf], check=True)
        return subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", elf],
                              check=True, capture_output=True, text=True).stdout


def main(obj, kname, min_mem=8):
    txt = disasm(obj)
    cur, ins = None, []
    for line in txt.splitlines():
        if line.endswith(">:") and "<" in line:
            cur = line[line.index("<") + 1:-2]
            continue
        if cur and kname in cur and line.startswith("\t"):
            m = re.match(r"\t(\S+)\s*(.*?)\s*//\s*([0-9A-Fa-f]+):", line)
            if m:
                ins.append((int(m.group(3), 16), m.group(1), line))
    addr = [a for a, _, _ in ins]
    loops = []
    for i, (a, op, args) in enumerate(ins):
        if op.startswith("s_cbranch") or op == "s_branch":
            m = re.search(r"<[^>]*\+0x([0-9a-f]+)>", args)
            if not m:
                continue
            # target: llvm-objdump prints <symbol+0xoff>; the kernel symbol starts at addr[0]
            tgt = addr[0] + int(m.group(1), 16)
            if tgt <= a:
                loops.append((tgt, a))
    rows = []
    for lo, hi in set(loops):
        c = collections.Counter()
        n = waits = 0
        for a, op, line in ins:
            if lo <= a <= hi:
                n += 1
                mm = re.match(r"(scratch|global|buffer)_(load|store)_(\w+)", op)
                if mm:
                    c[mm.group(0)] += 1
                if op == "s_waitcnt" and "vmcnt" in line:
                    waits += 1
        mem = sum(c.values())
        if mem >= min_mem:
            rows.append((lo, hi, n, mem, waits, c))
    rows.sort(key=lambda r: (r[0], -r[1]))
    for lo, hi, n, mem, waits, c in rows:
        print("%06x-%06x %6d ins %4d mem %3d vmwait  %s" % (lo, hi, n, mem, waits,
              " ".join("%s:%d" % (k.replace("scratch_", "s_").replace("global_", "g_"), v)
                       for k, v in c.most_common(6))))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 8)
