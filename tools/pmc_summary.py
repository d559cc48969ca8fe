#!/usr/bin/env python3
"""Turn the rocprofv3 passes written by tools/prof_round.sh into the committed
profile summaries.

    python tools/pmc_summary.py gpurun_out/prof r01

For each workload (c2 -> pair, c3 -> batch, c5 -> slab on one GPU):
  * copies the kernel-trace stats and the FETCH_SIZE / WRITE_SIZE counter CSVs
    and the bench line to profiles/<round>_<cfg>_*;
  * writes profiles/pmc_<workload>.json, which bench.py reads for
    roofline.traffic: HBM bytes per launch of the dominant engine kernel.
    The counters were collected in separate --pmc passes, with no traces
    combined.  Corrections follow MI355X_MICROARCH.md, HBM section:
      - FETCH_SIZE counts half the bytes of 16-B/lane reads (the granule
        reads), so it is doubled;
      - WRITE_SIZE is exact for the 16-B/lane granule stores;
      - the 1-B/lane row reads are uncalibrated (< 1% of the total).
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ALGO_BYTES_PER_CELL = 12
CELLS = {"c2": 65536 * 65536, "c3": 1024 * 8192 * 8192, "c5": (1 << 20) * (1 << 20)}
WORKLOAD = {"c2": "pair", "c3": "batch", "c5": "slab"}


def _rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def _engine_kernel(rows, key="Kernel_Name"):
    names = [r[key] for r in rows if "swmi::" in r[key]]
    return max(set(names), key=names.count)


def per_launch(path):
    rows = _rows(path)
    k = _engine_kernel(rows)
    vals = [float(r["Counter_Value"]) for r in rows if r["Kernel_Name"] == k]
    return k, sum(vals) / len(vals), len(vals)


def main():
    src, rnd = sys.argv[1], sys.argv[2]
    prof = os.path.join(ROOT, "profiles")
    for cfg in ("c2", "c3", "c5"):
        stats = os.path.join(src, "kt_" + cfg, cfg + "_kernel_stats.csv")
        fetch = os.path.join(src, "fetch_" + cfg, cfg + "_counter_collection.csv")
        write = os.path.join(src, "write_" + cfg, cfg + "_counter_collection.csv")
        if not all(os.path.exists(p) for p in (stats, fetch, write)):
            print("skip", cfg)
            continue
        shutil.copy(stats, os.path.join(prof, "%s_%s_kernel_stats.csv" % (rnd, cfg)))
        shutil.copy(fetch, os.path.join(prof, "%s_%s_pmc_fetch.csv" % (rnd, cfg)))
        shutil.copy(write, os.path.join(prof, "%s_%s_pmc_write.csv" % (rnd, cfg)))
        bench = os.path.join(src, "bench_%s.json" % cfg)
        if os.path.exists(bench):
            shutil.copy(bench, os.path.join(prof, "%s_bench_%s.json" % (rnd, cfg)))
        k, fkb, nf = per_launch(fetch)
        k2, wkb, nw = per_launch(write)
        assert k == k2, (k, k2)
        st = [r for r in _rows(stats) if r["Name"] == k][0]
        read_raw = fkb * 1024
        out = {
            "kernel": k,
            "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes (MI355X_MICROARCH.md HBM "
                      "section); KB per dispatch averaged over %d/%d dispatches; FETCH_SIZE doubled for the 16-B/lane "
                      "granule reads (gfx950 reports half of a wide coalesced read); 1-B/lane row reads uncalibrated"
                      % (nf, nw),
            "kernel_avg_ns": float(st["AverageNs"]),
            "kernel_calls": int(st["Calls"]),
            "fetch_size_kb": fkb,
            "write_size_kb": wkb,
            "read_bytes_raw": read_raw,
            "read_bytes_corrected": 2 * read_raw,
            "write_bytes": wkb * 1024,
            "hbm_bytes_per_launch": 2 * read_raw + wkb * 1024,
            "algorithmic_bytes_per_launch": CELLS[cfg] * ALGO_BYTES_PER_CELL,
        }
        out["traffic_over_algorithmic"] = out["hbm_bytes_per_launch"] / out["algorithmic_bytes_per_launch"]
        with open(os.path.join(prof, "pmc_%s.json" % WORKLOAD[cfg]), "w") as f:
            json.dump(out, f, indent=1)
        print(cfg, json.dumps(out))


if __name__ == "__main__":
    main()
