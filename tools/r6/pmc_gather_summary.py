"""Per-kernel summary of tools/r6/pmc_gather.sh passes: counters per launch (mean over launches).
Usage: python tools/r6/pmc_gather_summary.py <dir> [kernel-substring ...]"""
import collections
import csv
import glob
import os
import sys


def load(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg


def main(d, pats):
    agg = load(d)
    for name, c in agg.items():
        if pats and not any(p in name for p in pats):
            continue
        print("==", name[:90])
        for k in sorted(c):
            v = c[k]
            print("  %-40s %14.4g  (n=%d)" % (k, sum(v) / len(v), len(v)))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:] or ["encode5", "sdf_kernel", "field_mlp"])
