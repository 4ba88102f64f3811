"""Copy a rocprofv3 output directory's summaries into gpurun_out, keeping only
the engine's kernels (mc::) in the per-dispatch CSVs (the full traces of a
bench run exceed gpurun's 64 MiB return limit).
    python scripts/prof_filter.py SRC_DIR DST_DIR"""
import csv
import os
import shutil
import sys

src, dst = sys.argv[1], sys.argv[2]
os.makedirs(dst, exist_ok=True)
for root, _, files in os.walk(src):
    for f in files:
        p = os.path.join(root, f)
        if not f.endswith(".csv"):
            continue
        out = os.path.join(dst, f)
        if "stats" in f:
            shutil.copy(p, out)
            continue
        with open(p, newline="") as fi, open(out, "w", newline="") as fo:
            r = csv.reader(fi)
            w = csv.writer(fo)
            hdr = next(r, None)
            if hdr is None:
                continue
            w.writerow(hdr)
            col = hdr.index("Kernel_Name") if "Kernel_Name" in hdr else None
            for row in r:
                if col is None or "mc::" in row[col]:
                    w.writerow(row)
