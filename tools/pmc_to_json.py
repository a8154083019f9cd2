"""Fold the two rocprofv3 HBM passes of a bench command (FETCH_SIZE and
WRITE_SIZE, run separately: MI355X_MICROARCH.md 'rocprofv3 PMC slots') into
profiles/pmc_traffic.json, which bench.py reads for roofline.traffic.

Corrections (MI355X_MICROARCH.md, HBM section): both counters are in KB
(x 1024); on gfx950 FETCH_SIZE tallies 128-B requests at 64 B, so it is
doubled.  Traffic per launch = the mean over the kernel's dispatches.

    python tools/pmc_to_json.py <fetch_dir> <write_dir> <key> <kernel-substring> [src] [grbm_dir]

grbm_dir (optional): a pass with GRBM_GUI_ACTIVE; the entry then also holds
the kernel's effective clock, GRBM_GUI_ACTIVE / 8 XCDs / dispatch time
(MI355X_MICROARCH.md 'DVFS give-back': within 3 % of the in-kernel clock on
dispatches of 10 ms or more), which bench.py's issue roofline uses.
"""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def mean_counter(d, name, ksub):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv")))
            if ksub in r["Kernel_Name"] and r["Counter_Name"] == name]
    if not vals:
        raise SystemExit(f"no {name} rows for {ksub} in {d}")
    return sum(vals) / len(vals), len(vals)


def main():
    fdir, wdir, key, ksub = sys.argv[1:5]
    src = sys.argv[5] if len(sys.argv) > 5 else f"{fdir} + {wdir}"
    gdir = sys.argv[6] if len(sys.argv) > 6 else None
    fkb, nf = mean_counter(fdir, "FETCH_SIZE", ksub)
    wkb, nw = mean_counter(wdir, "WRITE_SIZE", ksub)
    fetch = 2.0 * fkb * 1024.0
    write = wkb * 1024.0
    out_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    d = json.load(open(out_path)) if os.path.exists(out_path) else {}
    d[key] = {"hbm_bytes_per_launch": round(fetch + write), "fetch_bytes": round(fetch),
              "write_bytes": round(write), "fetch_size_kb_raw": fkb, "write_size_kb_raw": wkb,
              "dispatches": [nf, nw], "kernel": ksub, "source": src,
              "correction": "KB x 1024; FETCH_SIZE x 2 (gfx950 128-B requests tallied at 64 B)"}
    if gdir:
        clk = [float(r["Counter_Value"]) / 8.0 /
               ((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9) / 1e9
               for r in csv.DictReader(open(os.path.join(gdir, "run_counter_collection.csv")))
               if ksub in r["Kernel_Name"] and r["Counter_Name"] == "GRBM_GUI_ACTIVE"]
        if clk:
            d[key]["effective_clock_ghz"] = round(sum(clk) / len(clk), 3)
            d[key]["clock_source"] = f"GRBM_GUI_ACTIVE / 8 / dispatch time ({gdir}, {len(clk)} dispatches)"
    json.dump(d, open(out_path, "w"), indent=1, sort_keys=True)
    print(key, d[key])


if __name__ == "__main__":
    main()
