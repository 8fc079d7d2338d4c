"""Summarise rocprofv3 PMC passes (tools/gpu_pmc.sh output) per kernel.

usage: python tools/pmc_summary.py gpurun_out/pmc > profiles/rNN_pmc_summary.md
       [--traffic-json profiles/traffic_rNN.json]

Each pass directory holds run_counter_collection.csv (one row per dispatch x
counter).  Values are averaged per dispatch of each kernel.  HBM bytes follow
MI355X_MICROARCH.md "HBM/rocprofv3": FETCH_SIZE is in KiB and on gfx950 reports
half of the bytes of wide streaming reads, so fetch bytes = 2 * 1024 * FETCH_SIZE
(an upper bound for narrower access patterns); WRITE_SIZE = 1024 * WRITE_SIZE.
"""
import argparse
import collections
import csv
import glob
import json
import os


def short(name):
    return name.split("(")[0].replace("void ", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir")
    ap.add_argument("--traffic-json", default=None)
    a = ap.parse_args()
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(a.pmc_dir, "*", "run_counter_collection.csv"))):
        seen = set()
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = short(r["Kernel_Name"])
                acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                key = (f, r["Dispatch_Id"])
                if key not in seen:
                    seen.add(key)
                    dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print("# PMC summary (per dispatch averages; durations include PMC overhead)\n")
    kernels = sorted(acc, key=lambda k: -sum(dur[k]) / max(len(dur[k]), 1))
    traffic = {}
    for k in kernels:
        if k.startswith("__amd"):
            continue
        d = dur[k]
        print(f"## {k}  (dispatches {len(d)}, mean {sum(d) / len(d):.1f} us)\n")
        print("| counter | mean per dispatch |\n|---|---|")
        for c in sorted(acc[k]):
            v = acc[k][c]
            print(f"| {c} | {sum(v) / len(v):.6g} |")
        m = {c: sum(v) / len(v) for c, v in acc[k].items()}
        if "FETCH_SIZE" in m:
            fb = 2 * 1024 * m["FETCH_SIZE"]
            print(f"| hbm_read_bytes (2*1024*FETCH_SIZE) | {fb:.6g} |")
            traffic[k] = {"read_bytes": fb}
        if "WRITE_SIZE" in m:
            wb = 1024 * m["WRITE_SIZE"]
            print(f"| hbm_write_bytes (1024*WRITE_SIZE) | {wb:.6g} |")
            traffic.setdefault(k, {})["write_bytes"] = wb
        if "SQ_WAVE_CYCLES" in m and m.get("SQ_WAVE_CYCLES"):
            for c in ("SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY"):
                if c in m:
                    print(f"| {c}/SQ_WAVE_CYCLES | {m[c] / m['SQ_WAVE_CYCLES']:.3f} |")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and m.get("GRBM_GUI_ACTIVE"):
            # busy cycles are summed over 256 CUs x 4 SIMDs; GRBM_GUI_ACTIVE is
            # summed over the 8 XCDs, so the kernel's cycles are GUI_ACTIVE / 8
            print(f"| MFMA busy frac (MFMA_BUSY / (GUI_ACTIVE/8 * 1024)) | "
                  f"{m['SQ_VALU_MFMA_BUSY_CYCLES'] / (m['GRBM_GUI_ACTIVE'] / 8 * 1024):.3f} |")
        print()
    if a.traffic_json:
        out = {}
        for k, t in traffic.items():
            if k.startswith("knn_screen16_kernel") or k.startswith("knn_screen_kernel"):
                out["knn_screen_bytes_per_launch"] = t.get("read_bytes", 0) + t.get("write_bytes", 0)
            out[k] = t
        with open(a.traffic_json, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
