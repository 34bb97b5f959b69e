#!/usr/bin/env python3
"""Per-source-line memory map of one kernel: disassembly with line info
(llvm-objdump -d -l of a device ELF compiled with -gline-tables-only) ->
for every file:line, the scratch / global loads and stores and the vmcnt
waits attributed to it, sorted by count.  Finds the lines whose private-
segment traffic is a run-time-indexed array or a spill.

  python tools/line_map.py kdbg.dis k_enc_anaILi1 [file-substring] [top]
"""
import collections
import re
import sys


def main(dis, kname, fsub="", top=60):
    cur_k, line = None, "?"
    c = collections.defaultdict(collections.Counter)
    for ln in open(dis):
        if ln.endswith(">:\n") and "<" in ln:
            cur_k = ln[ln.index("<") + 1:-3]
            continue
        if not cur_k or kname not in cur_k:
            continue
        if ln.startswith("; /"):
            line = ln[2:].strip().rsplit("/", 1)[-1]
            continue
        m = re.match(r"\s+(\S+)", ln)
        if not m:
            continue
        op = m.group(1)
        mm = re.match(r"(scratch|global|buffer)_(load|store)", op)
        if mm:
            c[line][mm.group(1) + "_" + mm.group(2)] += 1
        elif op == "s_waitcnt" and "vmcnt" in ln:
            c[line]["wait_vm"] += 1
        c[line]["insts"] += 1
    rows = [(k, v) for k, v in c.items() if fsub in k]
    rows.sort(key=lambda kv: -(kv[1]["scratch_load"] + kv[1]["scratch_store"]))
    for k, v in rows[:top]:
        print("%-28s insts %5d  sl %4d ss %4d gl %4d gs %3d wait %4d" % (
            k, v["insts"], v["scratch_load"], v["scratch_store"], v["global_load"],
            v["global_store"], v["wait_vm"]))


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], a[1], a[2] if len(a) > 2 else "", int(a[3]) if len(a) > 3 else 60)
