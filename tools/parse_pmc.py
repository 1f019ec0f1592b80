#!/usr/bin/env python3
"""Summarise the rocprofv3 passes of tools/profile.sh for the bench's render kernel.

HBM bytes per launch follow MI355X_MICROARCH.md §HBM / cdna_hip_programming.md §7:
FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports exactly half the
bytes of wide (16 B/lane) coalesced reads, so the read side is doubled:
    hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024
The uncorrected figure is kept beside it.  FETCH_SIZE also counts Infinity-Cache
(MALL) hits, so it is an upper bound on DRAM reads.

The summary records the library build id (sha of the sources, mpiv_build_id), the
kernel, views per launch and MPI shape; bench.py uses it only when all of them match
the build it runs (load_pmc).  Run it in the tree whose sources were profiled.
"""
import csv
import glob
import json
import os
import shutil
import sys

KERNEL = "render_packed_kernel"  # override: argv[3]


def rows(path_glob):
    out = []
    for f in glob.glob(path_glob, recursive=True):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


def per_dispatch(counter_rows, name):
    vals = {}
    for r in counter_rows:
        if KERNEL in r.get("Kernel_Name", "") and r.get("Counter_Name") == name:
            vals.setdefault(r["Dispatch_Id"], 0.0)
            vals[r["Dispatch_Id"]] += float(r["Counter_Value"])
    return list(vals.values())


def main():
    global KERNEL
    out_dir, tag = sys.argv[1], sys.argv[2]
    if len(sys.argv) > 3:
        KERNEL = sys.argv[3]
    views = int(sys.argv[4]) if len(sys.argv) > 4 else 125
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prof = os.path.join(repo, "profiles")
    os.makedirs(prof, exist_ok=True)
    sys.path.insert(0, repo)
    from mpi_vision_amd import _lib
    res = {"kernel": KERNEL, "tag": tag, "views": views, "shape": [1024, 1024, 128],
           "build_id": _lib.source_hash(),
           "command": "python bench.py --steps 2 --warmup 1 --no-extras (tools/profile.sh)"}
    stats = glob.glob(os.path.join(out_dir, "trace", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(prof, f"{tag}_kernel_stats.csv"))
        for r in csv.DictReader(open(stats[0])):
            if KERNEL in r["Name"]:
                res["trace_calls"] = int(r["Calls"])
                res["trace_avg_ns"] = float(r["AverageNs"])
    fetch = per_dispatch(rows(os.path.join(out_dir, "FETCH_SIZE", "**", "*counter_collection.csv")), "FETCH_SIZE")
    write = per_dispatch(rows(os.path.join(out_dir, "WRITE_SIZE", "**", "*counter_collection.csv")), "WRITE_SIZE")
    hm = rows(os.path.join(out_dir, "TCC_HIT_sum_TCC_MISS_sum", "**", "*counter_collection.csv"))
    hit, miss = per_dispatch(hm, "TCC_HIT_sum"), per_dispatch(hm, "TCC_MISS_sum")
    if fetch and write:
        f = sum(fetch) / len(fetch)
        w = sum(write) / len(write)
        res.update(fetch_size_kib=f, write_size_kib=w, dispatches=len(fetch),
                   hbm_bytes_per_launch=(2 * f + w) * 1024, hbm_bytes_per_launch_uncorrected=(f + w) * 1024)
    if hit and miss:
        res["l2_hit_rate"] = sum(hit) / (sum(hit) + sum(miss))
    vrows = rows(os.path.join(out_dir, "VALU", "**", "*counter_collection.csv"))
    valu, gui = per_dispatch(vrows, "SQ_INSTS_VALU"), per_dispatch(vrows, "GRBM_GUI_ACTIVE")
    if valu and gui:
        # VALU issue capacity: 1024 SIMDs x one wave64 instruction per 2 cycles; GRBM_GUI_ACTIVE
        # sums the 8 XCDs' busy cycles
        cycles = sum(gui) / len(gui) / 8
        res["valu_insts_per_launch"] = sum(valu) / len(valu)
        res["valu_issue_frac"] = res["valu_insts_per_launch"] / (512 * cycles)
    trows = rows(os.path.join(out_dir, "TA", "**", "*counter_collection.csv"))
    ta, tgui = per_dispatch(trows, "TA_BUSY_avr"), per_dispatch(trows, "GRBM_GUI_ACTIVE")
    if ta and tgui:
        # TA_BUSY_avr: busy cycles averaged over the TA instances; GRBM_GUI_ACTIVE sums 8 XCDs
        res["ta_busy_frac"] = (sum(ta) / len(ta)) / (sum(tgui) / len(tgui) / 8)
    for name in (f"{tag}_render_pmc.json", "render_pmc.json"):
        with open(os.path.join(prof, name), "w") as fh:
            json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
