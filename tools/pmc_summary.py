"""Summarise rocprofv3 --pmc passes (tools/pmc.sh) into per-kernel HBM bytes per launch.

Corrections per MI355X_MICROARCH.md §HBM: FETCH_SIZE is in KiB and reports half the bytes of
wide (16 B/lane) coalesced reads on gfx950, so it is doubled; WRITE_SIZE (KiB) is exact for
16 B/lane stores and float atomics.  Gathers narrower than a line are uncalibrated (the SDF
kernel's hash-table reads): they are reported as measured x2, with a note.

Usage: python tools/pmc_summary.py gpurun_out/pmc profiles/r1/pmc_summary.json
"""
import collections
import csv
import json
import os
import sys


def _load(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    with open(path) as f:
        for r in csv.DictReader(f):
            agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg


def short(name):
    """Kernel symbol -> the C-ABI call bench.py times (kernel table names)."""
    table = [("rgb_fwd_kernel", "mli_rgb_fwd"), ("rgb_bwd_kernel", "mli_rgb_bwd"),
             ("dw4_partial_kernel", "mli_dw4"), ("dw4_reduce_kernel", "mli_dw4:reduce"),
             ("wgrad_kernel<256, 256", "mli_wgrad:big"), ("wgrad_dma_kernel<256, 256", "mli_wgrad:big"), ("wgrad_kernel<256, 320", "mli_wgrad:wide"),
             ("wgrad_kernel<32, 256", "mli_wgrad:thin"), ("wgrad_dma_kernel<256, 320", "mli_wgrad:wide"),
             ("wgrad_frag_kernel<256, 256", "mli_wgrad:big"), ("wgrad_frag_kernel<256, 320", "mli_wgrad:wide"),
             ("wgrad_frag_kernel<32, 256", "mli_wgrad:thin"), ("encode5_kernel", "mli_sdf:field/encode5"),
             ("field_mlp_kernel", "mli_sdf:field/mlp"), ("sdf_kernel", "mli_sdf:sdf"), ("sample_fine_kernel", "mli_sample_fine"),
             ("composite_fwd_kernel", "mli_composite_fwd"), ("composite_bwd_kernel", "mli_composite_bwd"),
             ("composite_loss_kernel", "mli_composite_loss"), ("composite_loss_finalize", "mli_composite_loss:finalize"),
             ("adamw_kernel", "mli_adamw"), ("pack_kernel", "mli_pack")]
    for key, val in table:
        if key in name:
            return val
    return None


def main(src, dst):
    fetch = _load(os.path.join(src, "fetch", "run_counter_collection.csv"))
    write = _load(os.path.join(src, "write", "run_counter_collection.csv"))
    l2 = _load(os.path.join(src, "l2", "run_counter_collection.csv"))
    out = {}
    for name, c in fetch.items():
        key = short(name)
        if key is None:
            continue
        fs = c["FETCH_SIZE"]
        ws = write.get(name, {}).get("WRITE_SIZE", [0.0])
        h = l2.get(name, {})
        hit, miss = sum(h.get("TCC_HIT_sum", [0.0])), sum(h.get("TCC_MISS_sum", [0.0]))
        rd = 2 * 1024 * sum(fs) / len(fs)
        wr = 1024 * sum(ws) / len(ws)
        out[key] = {"hbm_read_bytes": rd, "hbm_write_bytes": wr, "hbm_bytes": rd + wr,
                    "l2_hit_rate": hit / max(1.0, hit + miss), "launches": len(fs), "kernel": name}
    out["_note"] = ("per launch; FETCH_SIZE x2 (gfx950 16 B/lane correction) + WRITE_SIZE; narrow gathers "
                    "(mli_sdf hash-table reads) are uncalibrated")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    for k, v in sorted(out.items()):
        if not k.startswith("_"):
            print("%-20s read %8.1f MB  write %8.1f MB  L2 hit %.2f" % (k, v["hbm_read_bytes"] / 1e6,
                                                                      v["hbm_write_bytes"] / 1e6, v["l2_hit_rate"]))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
