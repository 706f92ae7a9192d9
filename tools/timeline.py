"""Per-step timeline of a rocprofv3 kernel trace (bench.py training run): which kernels run on
which stream, when, and what overlaps.  Usage: python tools/timeline.py <run_kernel_trace.csv> [step]"""
import csv
import sys

SHORT = [("rgb_fwd", "fwd"), ("rgb_bwd", "bwd"), ("wgrad_kernel<256, 256", "BIG"), ("wgrad_dma_kernel<256, 256", "BIG"),
         ("wgrad_frag_kernel<256, 256", "BIG"), ("wgrad_frag_kernel<256, 320", "WIDE"), ("wgrad_frag_kernel<32", "THIN"),
         ("wgrad_dma", "WIDE"),
         ("wgrad_kernel<32", "THIN"), ("encode5", "enc5"), ("field_mlp", "fmlp"), ("sdf_kernel", "sdf"),
         ("sample_fine", "fine"), ("sample_coarse", "coarse"), ("composite_loss_kernel", "cl"),
         ("composite_loss_finalize", "clfin"), ("composite_fwd", "cfwd"), ("dw4_partial", "dw4p"),
         ("dw4_reduce", "dw4r"), ("assemble", "asm"), ("adamw", "adam"), ("pack_kernel", "pack"),
         ("row_scale", "rowsc"), ("rays_kernel", "rays"), ("ray_batch", "batch"), ("copyBuffer", "copy"),
         ("elementwise", "fill"), ("distribution", "rand"), ("field_kernel", "field")]


def short(n):
    for k, v in SHORT:
        if k in n:
            return v
    return n[:20]


def main(path, step=50):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    fwd = [i for i, r in enumerate(rows) if "rgb_fwd" in r["Kernel_Name"]]
    i0, i1 = fwd[step], fwd[step + 1]
    t0 = int(rows[i0]["Start_Timestamp"])
    # include kernels that started up to 1.5 ms before this step's forward (the prefetch)
    sel = [r for r in rows if t0 - 1500000 <= int(r["Start_Timestamp"]) < int(rows[i1]["Start_Timestamp"])]
    for r in sel:
        s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
        print("%8.1f %8.1f %7.1f  q%-3s %s" % (s, e, e - s, r["Queue_Id"], short(r["Kernel_Name"])))
    print("step span (fwd to fwd): %.1f us" % ((int(rows[i1]["Start_Timestamp"]) - t0) / 1e3))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 50)
