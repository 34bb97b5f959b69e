#!/usr/bin/env python3
"""Table of tools/gpu_ko_pmc.sh results: per variant the analysis launch ms
and k_enc_ana<1>'s memory-pipeline counters per wave; the stage's price is
the product row minus the knockout row.
  python tools/ko_pmc_table.py gpurun_out/<tag> cur ko_bpvc ..."""
import json
import sys


def main(d, variants):
    cols = ("TCP_TOTAL_CACHE_ACCESSES_sum", "TD_TD_BUSY_sum", "TA_TA_BUSY_sum", "SQ_INSTS_VMEM_RD",
            "SQ_INSTS_VMEM_WR", "SQ_WAVE_CYCLES")
    print("%-12s %8s " % ("variant", "ana_ms") + " ".join("%12s" % c.replace("_sum", "")[-12:] for c in cols)
          + "   (per wave)")
    for v in variants:
        try:
            t = open("%s/dump_%s.txt" % (d, v)).read()
            sec = t.split("[k_enc_ana<1>]")[1].split("\n[")[0]
            val = {l.split()[0]: float(l.split()[1]) for l in sec.strip().splitlines()
                   if not l.strip().startswith("=")}
            ms = json.load(open("%s/%s.json" % (d, v)))["roofline"]["kernel_ms"]
        except Exception as e:  # noqa: BLE001
            print(v, "missing:", e)
            continue
        w = val.get("SQ_WAVES", 4096.0)
        print("%-12s %8.2f " % (v, ms) + " ".join("%12.0f" % (val.get(c, 0) / w) for c in cols))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
