#!/usr/bin/env python3
"""Knockout table of the lane analysis (tools/gpu_r04_ko.sh output) ->
profiles/<name>.json: per variant the analysis launch's kernel time and,
from the PMC passes, HBM bytes and wave stalls per k_enc_ana<1> launch;
each stage's price = product build minus the build without it.

  python tools/ko_summary.py gpurun_out/<tag> profiles/r04_ko_traffic.json cur bpvc ...
"""
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import pmc_means  # noqa: E402

KERNEL = "k_enc_ana<1>"


def pmc(src, pat):
    out = {}
    for db in glob.glob(os.path.join(src, pat, "*_results.db")):
        for k, d in pmc_means(db).items():
            out.setdefault(k, {}).update(d)
    return out


def main():
    src, dst, variants = sys.argv[1], sys.argv[2], sys.argv[3:]
    rows = {}
    for v in variants:
        line = json.load(open(os.path.join(src, v + ".json")))
        roof = line["roofline"]
        r = {"ms_per_step": line["ms_per_step"], "analysis_launch_ms": roof["kernel_ms"],
             "k_enc_npp_ms": roof["kernels"][1]["kernel_ms"]}
        p = pmc(src, "pmc_f_" + v)
        p.update({k: {**p.get(k, {}), **d} for k, d in pmc(src, "pmc_w_" + v).items()})
        d = p.get(KERNEL, {})
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            r["fetch_GB"] = d["FETCH_SIZE"] * 1024 / 1e9
            r["write_GB"] = d["WRITE_SIZE"] * 1024 / 1e9
            r["hbm_GB"] = r["fetch_GB"] + r["write_GB"]
        if "SQ_WAIT_ANY" in d and "SQ_WAVE_CYCLES" in d:
            r["wait_any_frac"] = d["SQ_WAIT_ANY"] / d["SQ_WAVE_CYCLES"]
        if "SQ_INSTS_VALU" in d and "SQ_WAVES" in d:
            r["valu_per_wave"] = d["SQ_INSTS_VALU"] / d["SQ_WAVES"]
            r["salu_per_wave"] = d.get("SQ_INSTS_SALU", 0) / d["SQ_WAVES"]
        rows[v] = r
    base = rows.get("cur")
    price = {}
    if base:
        for v, r in rows.items():
            if v == "cur":
                continue
            price[v] = {"ms": base["analysis_launch_ms"] - r["analysis_launch_ms"]}
            if "hbm_GB" in r and "hbm_GB" in base:
                price[v]["hbm_GB"] = base["hbm_GB"] - r["hbm_GB"]
    out = {"source": src, "kernel": KERNEL, "channels": 262144,
           "note": "ko_<stage>: k_ana.hip built with -DMELPE_KO_<STAGE> (encoder.h), the stage "
                   "skipped; its price is the product build minus the knockout. 'analysis' skips "
                   "all of analysis() (record copies and launch overhead remain).",
           "variants": rows, "price": price}
    json.dump(out, open(dst, "w"), indent=1)
    for v, r in rows.items():
        print(v, {k: round(x, 3) for k, x in r.items()})
    print("price", json.dumps(price))


if __name__ == "__main__":
    main()
