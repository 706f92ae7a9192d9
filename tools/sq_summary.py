"""Summarise tools/pmc_trio.sh passes into per-kernel SQ / MFMA / HBM figures per launch.

Units (MI355X_MICROARCH.md): SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* / SQ_BUSY_CYCLES count
quad-cycles; SQ_VALU_MFMA_BUSY_CYCLES counts cycles summed over SIMDs (32 per 32x32x16 MFMA);
GRBM_GUI_ACTIVE is summed over the 8 XCDs; FETCH_SIZE (KiB) is half the bytes of 16 B/lane
reads on gfx950 (x2), WRITE_SIZE (KiB) exact.  Derived per kernel:
  clock_ghz   = GRBM_GUI_ACTIVE / 8 / duration      (effective clock under the profiler)
  mfma_util   = SQ_VALU_MFMA_BUSY_CYCLES / (duration * clock * 1024 SIMDs)
  wait_frac   = SQ_WAIT_ANY / SQ_WAVE_CYCLES        (waves parked on s_waitcnt / barrier)
  issue_stall = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES   (waves stalled at issue)
  active_frac = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
Usage: python tools/sq_summary.py gpurun_out/pmc_trio profiles/r4/trio_pmc.json
"""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import short  # noqa: E402


def _counters(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg


def _durations(d):
    agg = collections.defaultdict(list)
    for path in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                agg[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return agg


def main(src, dst):
    kern = collections.defaultdict(dict)
    dur = collections.defaultdict(list)
    for p in sorted(glob.glob(os.path.join(src, "p*"))):
        if not os.path.isdir(p):
            continue
        for name, cs in _counters(p).items():
            for c, vals in cs.items():
                kern[name][c] = sum(vals) / len(vals)
        for name, ds in _durations(p).items():
            dur[name] += ds
    out = {}
    for name, c in kern.items():
        key = short(name) or name[:60]
        if not dur.get(name):
            continue
        t = sum(dur[name]) / len(dur[name]) * 1e-9
        rec = {"kernel": name, "duration_ms_profiled": round(t * 1e3, 4)}
        rec.update({k: v for k, v in sorted(c.items())})
        wc = c.get("SQ_WAVE_CYCLES")
        if c.get("GRBM_GUI_ACTIVE"):
            clk = c["GRBM_GUI_ACTIVE"] / 8 / t
            rec["clock_ghz"] = round(clk / 1e9, 3)
            if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
                rec["mfma_util"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (t * clk * 1024), 4)
        if wc:
            for k, n in (("SQ_WAIT_ANY", "wait_frac"), ("SQ_WAIT_INST_ANY", "issue_stall_frac"),
                         ("SQ_ACTIVE_INST_ANY", "active_frac"), ("SQ_ACTIVE_INST_VALU", "valu_frac"),
                         ("SQ_ACTIVE_INST_LDS", "lds_frac")):
                if k in c:
                    rec[n] = round(c[k] / wc, 4)
        if "FETCH_SIZE" in c:
            rec["hbm_read_bytes"] = 2 * 1024 * c["FETCH_SIZE"]
        if "WRITE_SIZE" in c:
            rec["hbm_write_bytes"] = 1024 * c["WRITE_SIZE"]
        if "hbm_read_bytes" in rec and "hbm_write_bytes" in rec:
            rec["hbm_tb_s_profiled"] = round((rec["hbm_read_bytes"] + rec["hbm_write_bytes"]) / t / 1e12, 3)
        out.setdefault(key, rec)
    out["_note"] = __doc__.split("Usage")[0].strip()
    with open(dst, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    for k, v in sorted(out.items(), key=lambda kv: -kv[1].get("duration_ms_profiled", 0) if isinstance(kv[1], dict) else 0):
        if k.startswith("_"):
            continue
        print("%-26s %7.3f ms  mfma %s  wait %s  stall %s  active %s  clk %s" % (
            k, v["duration_ms_profiled"], v.get("mfma_util"), v.get("wait_frac"), v.get("issue_stall_frac"),
            v.get("active_frac"), v.get("clock_ghz")))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
