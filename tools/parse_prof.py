#!/usr/bin/env python3
"""Summarise tools/profile.sh's rocprofv3 passes per (kernel, grid size).

    python tools/parse_prof.py gpurun_out/prof <tag>

Every libmpiv dispatch of the profiled bench.py run is grouped by its kernel name
(template arguments included, as mpiv_route reports it) and its grid size in work-items, and
again per bench phase tag: bench.py launches a marker kernel (mpiv_mark) before each timed region,
and every later dispatch belongs to the last marker's tag (configs.PROF_TAGS), which separates
sub-legs that launch the same kernel and grid (the backward with and without checkpoints, in plane
groups; config 3's drop-in and its timed launches).  Entries without "tag" aggregate every dispatch
of that kernel and grid.  Per group:
rocprof's call count and average / min / max duration (kernel-trace pass) and, from the
separate --pmc passes, per-dispatch averages of

    hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024

(MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are KiB; on gfx950 FETCH_SIZE
reports half the bytes of wide 16-B/lane reads, so the read side is doubled; Infinity
Cache hits are counted, so it bounds DRAM reads from above; the uncorrected sum is kept
beside it), the L2 hit rate, VALU issue and TA busy fractions.

Writes profiles/<tag>_prof_summary.json and profiles/prof_summary.json (bench.py quotes
the latter only when its build id equals the library it runs) and copies the raw
kernel-stats CSV to profiles/<tag>_kernel_stats.csv.  Run it in the tree whose sources
were profiled.
"""
import csv
import glob
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short_name(full: str) -> str:
    """'void mpiv::render_rows_kernel<false, 6, true, false, 3, false, false>(HIP_vector_type...)' ->
    'render_rows_kernel<false, 6, true, false, 3, false, false>'."""
    s = full.strip()
    if s.startswith("void "):
        s = s[5:]
    depth = 0
    for i, ch in enumerate(s):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            s = s[:i]
            break
    return s[len("mpiv::"):] if s.startswith("mpiv::") else s


def rows(path_glob):
    out = []
    for f in sorted(glob.glob(path_glob, recursive=True)):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


def _tagged(rows, grid_of):
    """(row, tag) for every libmpiv dispatch in submission order (Dispatch_Id): the tag is the name
    of the last mark_kernel dispatched before it (bench.py phase markers, grid = tag x 64), None
    before the first marker."""
    from mpi_vision_amd.configs import PROF_TAGS
    names = {v: k for k, v in PROF_TAGS.items()}
    tag = None
    for r in sorted(rows, key=lambda r: int(r["Dispatch_Id"])):
        name = r.get("Kernel_Name", "")
        if "mpiv::" not in name:
            continue
        if "mark_kernel" in name:
            tag = names.get(grid_of(r) // 64)
            continue
        yield r, tag


def trace_groups(trace_rows):
    """{(kernel, grid, tag): [duration ns]} plus the untagged aggregate {(kernel, grid, None): ...}."""
    g = {}
    grid_of = lambda r: int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])  # noqa: E731
    for r, tag in _tagged(trace_rows, grid_of):
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        k = (short_name(r["Kernel_Name"]), grid_of(r))
        g.setdefault(k + (None,), []).append(d)
        if tag is not None:
            g.setdefault(k + (tag,), []).append(d)
    return g


def counter_groups(counter_rows):
    """{(kernel, grid, tag): {counter: [per-dispatch value]}} (tag None: every dispatch)"""
    per = {}
    # one row per (dispatch, counter): the marker logic needs one row per dispatch, so tag the
    # dispatch ids first
    first = {}
    for r in counter_rows:
        first.setdefault(r["Dispatch_Id"], r)
    tags = {r["Dispatch_Id"]: t for r, t in _tagged(list(first.values()), lambda r: int(r["Grid_Size"]))}
    for r in counter_rows:
        if "mpiv::" not in r.get("Kernel_Name", "") or "mark_kernel" in r["Kernel_Name"]:
            continue
        k = (short_name(r["Kernel_Name"]), int(r["Grid_Size"]))
        tag = tags.get(r["Dispatch_Id"])
        for key in [k + (None,)] + ([k + (tag,)] if tag is not None else []):
            d = per.setdefault(key, {}).setdefault(r["Counter_Name"], {})
            d[r["Dispatch_Id"]] = d.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return {k: {c: list(v.values()) for c, v in cs.items()} for k, cs in per.items()}


def mean(x):
    return sum(x) / len(x) if x else None


def main():
    out_dir, tag = sys.argv[1], sys.argv[2]
    sys.path.insert(0, REPO)
    from mpi_vision_amd import _lib
    prof = os.path.join(REPO, "profiles")
    stats = glob.glob(os.path.join(out_dir, "trace", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(prof, f"{tag}_kernel_stats.csv"))
    tg = trace_groups(rows(os.path.join(out_dir, "trace", "**", "*kernel_trace.csv")))
    cg = {}
    for p in ("FETCH_SIZE", "WRITE_SIZE", "TCC_HIT_sum_TCC_MISS_sum", "VALU", "TA"):
        for k, cs in counter_groups(rows(os.path.join(out_dir, p, "**", "*counter_collection.csv"))).items():
            cg.setdefault(k, {}).update(cs)
    launches = []
    for key in sorted(set(tg) | set(cg), key=lambda k: (k[0], k[1], k[2] or "")):
        kern, grid, phase = key
        e = {"kernel": kern, "grid": grid}
        if phase is not None:
            e["tag"] = phase
        d = tg.get(key)
        if d:
            e.update(calls=len(d), avg_ns=mean(d), min_ns=min(d), max_ns=max(d))
        c = cg.get(key, {})
        f, w = mean(c.get("FETCH_SIZE", [])), mean(c.get("WRITE_SIZE", []))
        if f is not None and w is not None:
            e.update(fetch_kib=f, write_kib=w, hbm_bytes=(2 * f + w) * 1024, hbm_bytes_uncorrected=(f + w) * 1024,
                     pmc_dispatches=len(c["FETCH_SIZE"]))
        hit, miss = c.get("TCC_HIT_sum"), c.get("TCC_MISS_sum")
        if hit and miss:
            e["l2_hit_rate"] = sum(hit) / (sum(hit) + sum(miss))
        valu, gui = c.get("SQ_INSTS_VALU"), c.get("GRBM_GUI_ACTIVE")
        if valu and gui:
            # VALU issue capacity: 1024 SIMDs x one wave64 instruction per 2 cycles; GRBM_GUI_ACTIVE
            # sums the 8 XCDs' busy cycles
            e["valu_insts"] = mean(valu)
            e["valu_issue_frac"] = mean(valu) / (512 * mean(gui) / 8)
        ta = c.get("TA_BUSY_avr")
        if ta and gui:
            e["ta_busy_frac"] = mean(ta) / (mean(gui) / 8)
        launches.append(e)
    res = {"tag": tag, "build_id": _lib.source_hash(),
           "command": "tools/profile.sh: rocprofv3 --kernel-trace --stats, then one --pmc pass per counter group, "
                      "each over `python bench.py " + os.environ.get("PROF_ARGS_DESC", "(see tools/profile.sh)") + "`",
           "hbm_bytes_def": "(2*FETCH_SIZE + WRITE_SIZE) * 1024 per dispatch (gfx950 FETCH_SIZE halving corrected)",
           "launches": launches}
    for name in (f"{tag}_prof_summary.json", "prof_summary.json"):
        with open(os.path.join(prof, name), "w") as fh:
            json.dump(res, fh, indent=1)
    for e in launches:
        print(json.dumps(e))


if __name__ == "__main__":
    main()
