"""Summarise a stencil A/B directory (tools/stencil_ab_r5.sh layout):
python tools/stencil_ab_summary.py DIR -> per variant: residual / J.x kernel
us (rocprofv3 average), FETCH_SIZE x 2 KB / the 2.147 GB read minimum at
8192^2, and the algorithmic fraction of 8 TB/s (48 B per cell)."""
import csv
import os
import sys

O = sys.argv[1]
MIN = 2 * 8192 * 8192 * 16
ALG = 48 * 8192 * 8192
for tag in sorted(os.listdir(O)):
    st = os.path.join(O, tag, "stats", "run_kernel_stats.csv")
    fe = os.path.join(O, tag, "fetch", "run_counter_collection.csv")
    if not (os.path.exists(st) and os.path.exists(fe)):
        continue
    us = {}
    for r in csv.DictReader(open(st)):
        for k in ("residual_kernel", "jvp_kernel"):
            if k in r["Name"]:
                us[k] = float(r["AverageNs"]) / 1e3
    fv = {}
    for r in csv.DictReader(open(fe)):
        for k in ("residual_kernel", "jvp_kernel"):
            if k in r["Kernel_Name"]:
                fv.setdefault(k, []).append(float(r["Counter_Value"]))
    f = {k: sum(v) / len(v) * 2048 / MIN for k, v in fv.items()}
    print(f"{tag}: residual {us['residual_kernel']:.1f} us, J.x {us['jvp_kernel']:.1f} us; "
          f"fetch x {f['residual_kernel']:.3f} / {f['jvp_kernel']:.3f}; "
          f"frac {ALG / us['residual_kernel'] / 1e3 / 8000:.3f} / {ALG / us['jvp_kernel'] / 1e3 / 8000:.3f}")
