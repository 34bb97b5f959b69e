#!/usr/bin/env python3
"""Summarise rocprofv3 output databases (rocpd SQLite) into profiles/.

  python tools/prof_summary.py <gpurun_out dir> <tag> [channels]

Reads   <dir>/prof_kt/*_results.db        (--kernel-trace --stats pass)
        <dir>/pmc_*/*_results.db          (one --pmc pass each)
Writes  profiles/<tag>_kernel_stats.txt   per-kernel calls / total / average
        profiles/<tag>_pmc.txt            per-kernel counter means per dispatch
        profiles/pmc_latest.json          HBM bytes per kernel launch, one set
                                          per channel count (read by bench.py)

FETCH_SIZE / WRITE_SIZE are rocprofv3's derived counters in KiB per dispatch
(TCC_EA0_RDREQ / _WRREQ x request size).  MI355X_MICROARCH.md: on gfx950
FETCH_SIZE under-reports wide (16 B/lane) coalesced streaming reads by 2x;
the codec's accesses are 2-4 B per lane, an uncalibrated width, so the raw
value is reported and the correction is noted, not applied.
"""
import collections
import glob
import json
import os
import sqlite3
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    """demangled kernel name without its argument list and return type:
    'void k_enc_ana<1>(EncState*, ...)' -> 'k_enc_ana<1>'"""
    n = name.split("(")[0]
    return n[5:] if n.startswith("void ") else n


def is_codec(name):
    return short(name).startswith("k_")


def kernel_stats(db):
    c = sqlite3.connect(db)
    rows = list(c.execute("select name,total_calls,total_duration,average,percentage "
                          "from top_kernels"))
    return rows


def pmc_means(db):
    """mean counter values per dispatch of each kernel, leaving out each
    kernel's first dispatch when it has more than one: melpe_engine_create
    launches every codec kernel once at its full grid with no work (the
    scratch reservation), and that launch would dilute the means"""
    c = sqlite3.connect(db)
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for name, disp, cn, cv in c.execute(
            "select name,dispatch_id,counter_name,counter_value from pmc_events"):
        per[(short(name), disp)][cn] += cv
    first = {}
    for (k, disp) in per:
        first[k] = min(first.get(k, disp), disp)
    count = collections.Counter(k for (k, _) in per)
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for (k, disp), v in per.items():
        if count[k] > 1 and disp == first[k]:
            continue
        for cn, cv in v.items():
            agg[k][cn].append(cv)
    return {k: {cn: sum(v) / len(v) for cn, v in d.items()} for k, d in agg.items()}


def main():
    src, tag = sys.argv[1], sys.argv[2]
    prof = os.path.join(ROOT, "profiles")
    kt = glob.glob(os.path.join(src, "prof_kt", "*_results.db"))
    if kt:
        rows = kernel_stats(kt[0])
        with open(os.path.join(prof, tag + "_kernel_stats.txt"), "w") as f:
            f.write("# rocprofv3 --kernel-trace --stats (%s); durations in ms (rocpd top_kernels, us / 1e3)\n" % tag)
            f.write("%-22s %6s %14s %12s %7s\n" % ("kernel", "calls", "total_ms", "avg_ms", "pct"))
            for n, calls, tot, avg, pct in rows:
                f.write("%-22s %6d %14.1f %12.3f %7.2f\n" % (short(n)[:22], calls, tot / 1e3,
                                                           avg / 1e3, pct))
            # the bench's legs launch the same kernels at different sizes:
            # per launch size (grid_x = threads = channels, or waves x 64 for
            # the wave-per-channel kernels), so a leg's HIP-event average can
            # be checked against the trace
            f.write("\n# per launch size (grid_x threads); durations in ms\n")
            f.write("%-22s %10s %6s %12s %10s\n" % ("kernel", "grid_x", "calls", "total_ms", "avg_ms"))
            c = sqlite3.connect(kt[0])
            for n, gx, calls, tot in c.execute(
                    "select name, grid_x, count(*), sum(duration) from kernels "
                    "group by name, grid_x order by sum(duration) desc"):
                if not is_codec(n) or short(n).startswith("k_derive"):
                    continue
                f.write("%-22s %10d %6d %12.1f %10.3f\n" % (short(n)[:22], gx, calls, tot / 1e6,
                                                           tot / 1e6 / calls))
            # dispatch by dispatch for the short series (the bench's main
            # loop: W warmup then K timed steps, whose mean is its kernel_ms)
            f.write("\n# dispatches in order, series of <= 32 (ms)\n")
            for n, gx in list(c.execute("select name, grid_x from kernels "
                                        "group by name, grid_x having count(*) <= 32")):
                if not is_codec(n) or short(n).startswith(("k_derive", "k_reset", "k_synth_seed", "k_vad_reset",
                                        "k_modem_reset")):
                    continue
                d = [r[0] / 1e6 for r in c.execute("select duration from kernels where name = ? and "
                                                   "grid_x = ? order by start", (n, gx))]
                f.write("%-22s %10d %s\n" % (short(n)[:22], gx, " ".join("%.2f" % x for x in d)))
    pm = {}
    if len(sys.argv) <= 3:	# PMC summaries only with the channel count they were taken at
        return
    for db in sorted(glob.glob(os.path.join(src, "pmc_*", "*_results.db"))):
        for k, d in pmc_means(db).items():
            pm.setdefault(k, {}).update(d)
    if pm:
        with open(os.path.join(prof, tag + "_pmc.txt"), "w") as f:
            f.write("# rocprofv3 --pmc passes (%s): mean counter value per dispatch\n" % tag)
            for k in sorted(pm):
                if not k.startswith("k_enc") and k not in ("k_decode", "k_decode2"):
                    continue
                f.write("[%s]\n" % k)
                for cn in sorted(pm[k]):
                    f.write("  %-22s %20.1f\n" % (cn, pm[k][cn]))
                d = pm[k]
                if "SQ_WAVE_CYCLES" in d and "SQ_WAIT_ANY" in d:
                    f.write("  wait_any/wave_cycles   %20.3f\n" % (d["SQ_WAIT_ANY"] / d["SQ_WAVE_CYCLES"]))
                if "SQ_INSTS_VALU" in d and "SQ_WAVES" in d:
                    f.write("  valu_insts_per_wave    %20.1f\n" % (d["SQ_INSTS_VALU"] / d["SQ_WAVES"]))
        out = {"source": "profiles/%s_pmc.txt" % tag, "kernels": {},
               "channels": int(sys.argv[3]) if len(sys.argv) > 3 else None}
        for k, d in pm.items():
            if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
                out["kernels"][k] = {"fetch_bytes": d["FETCH_SIZE"] * 1024.0,
                                     "write_bytes": d["WRITE_SIZE"] * 1024.0,
                                     "bytes_per_launch": (d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024.0}
        # one set per channel count: a pass at another size keeps the others
        lp = os.path.join(prof, "pmc_latest.json")
        sets = []
        if os.path.exists(lp):
            old = json.load(open(lp))
            sets = old.get("sets", [old] if "kernels" in old else [])
        sets = [x for x in sets if x.get("channels") != out["channels"]] + [out]
        json.dump({"sets": sets}, open(lp, "w"), indent=1)


if __name__ == "__main__":
    main()
