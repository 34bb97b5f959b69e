#!/usr/bin/env python3
"""Per-kernel mean counter values per dispatch of rocprofv3 --pmc passes
(each directory one pass; the create-time reservation dispatch left out,
prof_summary.pmc_means), plus derived ratios where their counters are
present.

  python tools/pmc_dump.py <pass dir> [<pass dir> ...]
"""
import collections
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import pmc_means  # noqa: E402


def main(dirs):
    allk = collections.defaultdict(dict)
    for d in dirs:
        for db in glob.glob(os.path.join(d, "**", "*_results.db"), recursive=True):
            for k, v in pmc_means(db).items():
                allk[k].update(v)
    for k in sorted(allk):
        v = allk[k]
        print("[%s]" % k)
        for cn in sorted(v):
            print("  %-36s %20.1f" % (cn, v[cn]))
        r = {}
        if "SQ_INST_LEVEL_VMEM" in v and v.get("SQ_INSTS_VMEM"):
            r["vmem latency (quad-cycles per instr)"] = v["SQ_INST_LEVEL_VMEM"] / v["SQ_INSTS_VMEM"]
        if "TCP_TCC_READ_REQ_LATENCY_sum" in v and v.get("TCP_TCC_READ_REQ_sum"):
            r["L1->L2 read latency (cycles)"] = v["TCP_TCC_READ_REQ_LATENCY_sum"] / v["TCP_TCC_READ_REQ_sum"]
        if "TCP_TOTAL_CACHE_ACCESSES_sum" in v and "TCP_TCC_READ_REQ_sum" in v:
            r["L1 read misses / accesses"] = v["TCP_TCC_READ_REQ_sum"] / max(1.0, v["TCP_TOTAL_CACHE_ACCESSES_sum"])
        if "GRBM_GUI_ACTIVE" in v:
            for cn in ("TA_TA_BUSY_sum", "TD_TD_BUSY_sum", "TA_ADDR_STALLED_BY_TC_CYCLES_sum",
                       "TCP_PENDING_STALL_CYCLES_sum", "TCP_TCR_TCP_STALL_CYCLES_sum"):
                if cn in v:
                    r[cn + " / (GUI_ACTIVE x 256 CU)"] = v[cn] / (v["GRBM_GUI_ACTIVE"] / 8 * 256)
        for n, x in r.items():
            print("  = %-50s %10.3f" % (n, x))


if __name__ == "__main__":
    main(sys.argv[1:])
