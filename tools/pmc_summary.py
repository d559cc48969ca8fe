#!/usr/bin/env python3
"""Turn the rocprofv3 passes written by tools/prof_round.sh into the committed
profile summaries.

    python tools/pmc_summary.py gpurun_out/prof r02 [c2,c3a,...]

For each workload (c2 -> pair, c3 -> batch, c5 -> slab on one GPU, c5p8 -> slab_part: slab 0 of
C5's 8-way column split alone):
  * copies the kernel-trace stats, the counter CSVs and the bench line to
    profiles/<round>_<cfg>_*;
  * writes profiles/pmc_<workload>.json, which bench.py reads for its roofline,
    stamped with the sha256 of the libswmi355.so that was profiled (bench.py
    ignores a profile of another build).  Per launch of the dominant engine
    kernel, averaged over the profiled dispatches:
      - valu_insts_per_launch = SQ_INSTS_VALU (wave64 VALU instructions; the
        roofline counts 64 lane-ops each);
      - clock_ghz = GRBM_GUI_ACTIVE / 8 XCDs / kernel time (MI355X_MICROARCH.md,
        DVFS give-back);
      - hbm_bytes_per_launch = 2 x FETCH_SIZE + WRITE_SIZE (KB x 1024): gfx950
        FETCH_SIZE counts half the bytes of 16-B/lane reads (the granule
        reads), WRITE_SIZE is exact for the 16-B/lane granule stores; the
        1-B/lane row reads are uncalibrated (< 1 % of the total).
    Every counter group came from its own --pmc pass with nothing traced.
  * adds valu_mix: the fast / slow instruction-class fractions of the kernel's
    chunk loop (tools/issue_model.py, from a -save-temps compile of the same
    sources), which bench.py prices with the measured issue costs
    (profiles/r03_ubench_issue_classes.jsonl) for roofline.issue.

    python tools/pmc_summary.py --mix-only     # add / refresh valu_mix of the existing pmc_*.json
"""
import csv
import hashlib
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ALGO_BYTES_PER_CELL = 12
CELLS = {"c2": 65536 * 65536, "c3": 1024 * 8192 * 8192, "c5": (1 << 20) * (1 << 20),
         "c2a": 65536 * 65536, "c3a": 1024 * 8192 * 8192, "c5a": (1 << 20) * (1 << 20)}
# c2a / c3a / c5a: the same pairs with the affine constants (2, -3, 5, 2) (bench.py AFFINE_PARAMS)
WORKLOAD = {"c2": "pair", "c3": "batch", "c5": "slab", "c5p8": "slab_part", "c2a": "pair_affine", "c3a": "batch_affine",
            "c5a": "slab_affine"}


def cells(cfg):
    """Cells per launch; c5p8: slab 0 of the 8-way column split of C5 alone (bench.py --slab-of 8)."""
    if cfg == "c5p8":
        sys.path.insert(0, ROOT)
        import concurrentproject_amd as sw
        b = sw.slab_bounds(1 << 20, 1 << 20, 8, sw.SW_FLAG_DNA)
        return (b[1] - b[0]) * (1 << 20)
    return CELLS[cfg]
LIB = os.path.join(ROOT, "concurrentproject_amd", "libswmi355.so")


def _rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def _engine_kernel(rows, key="Kernel_Name"):
    names = [r[key] for r in rows if "swmi::" in r[key]]
    return max(set(names), key=names.count)


def per_launch(path, counter=None):
    """(kernel, mean counter value per dispatch, dispatches) of the engine kernel."""
    rows = _rows(path)
    k = _engine_kernel(rows)
    vals = [float(r["Counter_Value"]) for r in rows
            if r["Kernel_Name"] == k and (counter is None or r["Counter_Name"] == counter)]
    return k, sum(vals) / len(vals), len(vals)


def source_stamp():
    sys.path.insert(0, ROOT)
    import concurrentproject_amd as sw
    return sw.source_stamp()


def sha256(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        h.update(f.read())
    return h.hexdigest()


def valu_mix(kernel):
    """issue_model.kernel_mix of `kernel` (demangled name) from build/asm/<src>.s, compiled
    with the library's flags when missing or older than its source."""
    import subprocess
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import issue_model
    csrc = os.path.join(ROOT, "concurrentproject_amd", "csrc")
    base = "sw_flow3" if "sw_flow3" in kernel else "sw_flow2" if "sw_flow2_kernel" in kernel else "sw_kernels"
    out = os.path.join(ROOT, "build", "asm")
    s_path = os.path.join(out, base + "-hip-amdgcn-amd-amdhsa-gfx950.s")
    deps = [os.path.join(csrc, f) for f in (base + ".hip", "sw_device.h", "sw_internal.h")]
    if base == "sw_flow3":
        deps += [os.path.join(csrc, f) for f in ("sw_flow3_loops.inc", "sw_flow3r_loops.inc", "sw_flow3a_loops.inc",
                                                  "sw_flow3ra_loops.inc", "sw_flow3p_loops.inc", "sw_flow3r3_loops.inc")]
    if not os.path.exists(s_path) or os.path.getmtime(s_path) < max(os.path.getmtime(d) for d in deps):
        os.makedirs(out, exist_ok=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c",
                        "-save-temps", os.path.join(csrc, base + ".hip"), "-o", os.path.join(out, base + ".o")],
                       cwd=out, check=True, stderr=subprocess.DEVNULL)
    km = issue_model.kernel_mix(s_path, issue_model.mangled_filter(kernel))
    if km is None:
        return None
    km["source_sha256"] = source_stamp()
    km["method"] = "static census of the kernel's chunk loop (tools/issue_model.py kernel_mix)"
    return km


def mix_only():
    for wl in WORKLOAD.values():
        path = os.path.join(ROOT, "profiles", "pmc_%s.json" % wl)
        if not os.path.exists(path):
            continue
        out = json.load(open(path))
        out["valu_mix"] = valu_mix(out["kernel"])
        with open(path, "w") as f:
            json.dump(out, f, indent=1)
        print(wl, json.dumps(out["valu_mix"]))


def main():
    if sys.argv[1] == "--mix-only":
        return mix_only()
    src, rnd = sys.argv[1], sys.argv[2]
    only = sys.argv[3].split(",") if len(sys.argv) > 3 else None   # e.g. c3a,c5 (default: every pass present)
    prof = os.path.join(ROOT, "profiles")
    for cfg in ("c2", "c3", "c5", "c5p8", "c2a", "c3a", "c5a"):
        if only is not None and cfg not in only:
            continue
        stats = os.path.join(src, "kt_" + cfg, cfg + "_kernel_stats.csv")
        if not os.path.exists(stats):
            print("skip", cfg)
            continue
        if os.path.getmtime(stats) < os.path.getmtime(LIB):
            # the passes predate the library this would stamp them with (a failed or
            # older gpurun call left them): never label old counters with a new build
            sys.exit("%s is older than %s: re-run tools/prof_round.sh with this build" % (stats, LIB))
        shutil.copy(stats, os.path.join(prof, "%s_%s_kernel_stats.csv" % (rnd, cfg)))
        bench = os.path.join(src, "bench_%s.json" % cfg)
        if os.path.exists(bench):
            shutil.copy(bench, os.path.join(prof, "%s_bench_%s.json" % (rnd, cfg)))
        k = _engine_kernel(_rows(stats), key="Name")
        st = [r for r in _rows(stats) if r["Name"] == k][0]
        t_ns = float(st["AverageNs"])
        out = {"kernel": k, "lib_sha256": sha256(LIB), "source_sha256": source_stamp(), "kernel_avg_ns": t_ns,
               "kernel_calls": int(st["Calls"]),
               "algorithmic_bytes_per_launch": cells(cfg) * ALGO_BYTES_PER_CELL, "cells_per_launch": cells(cfg)}
        passes = []
        fetch = os.path.join(src, "fetch_" + cfg, cfg + "_counter_collection.csv")
        write = os.path.join(src, "write_" + cfg, cfg + "_counter_collection.csv")
        if os.path.exists(fetch) and os.path.exists(write):
            shutil.copy(fetch, os.path.join(prof, "%s_%s_pmc_fetch.csv" % (rnd, cfg)))
            shutil.copy(write, os.path.join(prof, "%s_%s_pmc_write.csv" % (rnd, cfg)))
            kf, fkb, nf = per_launch(fetch)
            kw, wkb, nw = per_launch(write)
            assert kf == kw == k, (kf, kw, k)
            out.update(fetch_size_kb=fkb, write_size_kb=wkb, read_bytes_corrected=2 * fkb * 1024,
                       write_bytes=wkb * 1024, hbm_bytes_per_launch=2 * fkb * 1024 + wkb * 1024)
            out["traffic_over_algorithmic"] = out["hbm_bytes_per_launch"] / out["algorithmic_bytes_per_launch"]
            passes.append("FETCH_SIZE (%d dispatches), WRITE_SIZE (%d)" % (nf, nw))
        sq = os.path.join(src, "sq_" + cfg, cfg + "_counter_collection.csv")
        if os.path.exists(sq):
            shutil.copy(sq, os.path.join(prof, "%s_%s_pmc_sq.csv" % (rnd, cfg)))
            names = sorted({r["Counter_Name"] for r in _rows(sq)})
            for c in names:
                kk, v, n = per_launch(sq, c)
                assert kk == k, (kk, k)
                out[c] = v
            out["valu_insts_per_launch"] = out.get("SQ_INSTS_VALU")
            out["valu_lane_ops_per_launch"] = out["valu_insts_per_launch"] * 64
            out["valu_frac_at_2p4ghz"] = out["valu_lane_ops_per_launch"] / (t_ns * 1e-9) / (256 * 4 * 32 * 2.4e9)
            out["valu_insts_per_cell"] = out["valu_insts_per_launch"] / cells(cfg)
            passes.append(" ".join(names))
        grbm = os.path.join(src, "grbm_" + cfg, cfg + "_counter_collection.csv")
        if os.path.exists(grbm):
            shutil.copy(grbm, os.path.join(prof, "%s_%s_pmc_grbm.csv" % (rnd, cfg)))
            kk, g, n = per_launch(grbm, "GRBM_GUI_ACTIVE")
            out["GRBM_GUI_ACTIVE"] = g
            out["clock_ghz"] = g / 8 / t_ns
            passes.append("GRBM_GUI_ACTIVE")
        out["valu_mix"] = valu_mix(k)
        out["method"] = ("rocprofv3 --pmc, one pass per group, nothing else traced: " + "; ".join(passes) +
                         "; kernel time from the --kernel-trace --stats run of the same command")
        with open(os.path.join(prof, "pmc_%s.json" % WORKLOAD[cfg]), "w") as f:
            json.dump(out, f, indent=1)
        print(cfg, json.dumps(out))


if __name__ == "__main__":
    main()
