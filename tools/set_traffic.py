"""HBM bytes per bootstrap of each stage of one launch set (tools/set_micro.py
under separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, as
tools/gpu_final_r6.sh runs them).

usage: python tools/set_traffic.py gpurun_out/<run>/pmc [--nb 8] [--merge profiles/traffic_r05.json]
                                   [--out profiles/traffic_r06.json]

read = 2 * 1024 * FETCH_SIZE (gfx950 correction, MI355X_MICROARCH.md
"HBM/rocprofv3"), write = 1024 * WRITE_SIZE.  A pass holds the table build
once and the launch set twice (set_micro's warm-up and timed repetition);
kernels are attributed to stages by name and the set's bytes are divided by
the set's bootstraps.
"""
import argparse
import collections
import csv
import glob
import json
import os


def stage(name):
    n = name.split("(")[0]
    if n.startswith("void "):
        n = n[5:]
    if n.startswith("sil_"):
        return "silhouette"
    if n.startswith(("snn_", "rs_")):
        return "snn"
    if n.startswith(("kb_", "kt_filter", "gather_rows")) or n in (
            "knn_fx_prep16_kernel<2, true>", "knn_fx_scan16_kernel<2, true>", "knn_fx_select_kernel<32>",
            "knn_fallback_merge_kernel", "knn_fallback_kernel<32, 20>"):
        return "knn_from_table"
    if n.startswith(("knn_", "kt_transpose")):
        return "knn_table"
    if n.startswith("scan_"):
        return "scan"
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir")
    ap.add_argument("--nb", type=int, default=8)
    ap.add_argument("--sets", type=int, default=2)
    ap.add_argument("--merge", default=None)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    tot = collections.defaultdict(float)
    for f in glob.glob(os.path.join(a.pmc_dir, "pass_*", "run_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            s = stage(r["Kernel_Name"])
            if s is None:
                continue
            c, v = r["Counter_Name"], float(r["Counter_Value"])
            if c == "FETCH_SIZE":
                tot[(s, "read")] += 2 * 1024 * v
            elif c == "WRITE_SIZE":
                tot[(s, "write")] += 1024 * v
    per = {}
    for (s, k), v in sorted(tot.items()):
        div = a.nb * a.sets if s != "knn_table" else 1
        per.setdefault(s, {})[k + "_bytes"] = v / div
    out = {}
    if a.merge:
        out = json.load(open(a.merge))
        out = {k: v for k, v in out.items() if k.startswith(("cocluster", "cof_tile", "knn_screen"))}
    for s, d in per.items():
        d["total_bytes"] = d.get("read_bytes", 0.0) + d.get("write_bytes", 0.0)
        out[f"set_stage_{s}" + ("_per_table_build" if s == "knn_table" else "_per_boot")] = d
    out["snn_bytes_per_boot"] = per["snn"]["total_bytes"] + per.get("scan", {}).get("total_bytes", 0.0)
    out["silhouette_bytes_per_boot"] = per["silhouette"]["total_bytes"]
    out["knn_from_table_bytes_per_boot"] = per["knn_from_table"]["total_bytes"]
    out["note"] = (f"round 6: tools/set_micro.py (one launch set of {a.nb} cfg3 bootstraps through "
                   "ccg_knn_boots_table_dev, the class-level SNN pass and ccg_silhouette_segments_dev) under "
                   "separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (tools/gpu_final_r6.sh); read = "
                   "2*1024*FETCH_SIZE (gfx950 correction), write = 1024*WRITE_SIZE; per bootstrap = the set's "
                   "bytes / the set's bootstraps (scans counted with SNN). Co-cluster and per-bootstrap screen "
                   "entries carried from round 5 (kernels unchanged).")
    txt = json.dumps(out, indent=1)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
