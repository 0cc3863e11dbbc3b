#!/usr/bin/env python3
"""Summarise rocprofv3 outputs into profiles/<tag>_*.{csv,json}.

    [PROFILE_OUT=dir] python tools/pmc_summary.py <tag> <trace_dir> <fetch_dir> <write_dir>

Per kernel: average duration (kernel trace) and HBM bytes per launch from the
separate FETCH_SIZE / WRITE_SIZE passes (units: KB).  On gfx950 FETCH_SIZE
counts half the bytes read (MI355X_MICROARCH.md §HBM for 16-B/lane streaming
loads; tools/probes/fetch_probe.hip measured the same 1/2 for 1-, 2-, 4- and
16-byte lanes: 1 GiB read -> 524298 KB, profiles/r03_probe_fetch_write.txt),
WRITE_SIZE the bytes written (256 MiB of 4-byte stores -> 262144 KB), so
hbm_bytes = 2 x FETCH_SIZE + WRITE_SIZE; the raw read figure is kept too.

The summary's "_meta" entry ties it to the build it profiled: the sha256 of
the libxylo_hip.so in this tree (the library the profiled bench loaded), the
tag and the creation time.  bench.py cites a summary's traffic only when its
library_sha256 equals the sha256 of the library the bench itself loaded.
"""
import collections
import csv
import datetime
import hashlib
import glob
import json
import os
import re
import shutil
import sys


def per_kernel(path, counter):
    agg = collections.defaultdict(list)
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def short(name):
    """'void xh::policy_train8_kernel<...>(...)' -> 'policy_train8_kernel',
    'xh::split::policy_train_split_kernel(...)' -> 'policy_train_split_kernel'."""
    m = re.match(r"(?:void )?(?:[A-Za-z_0-9]+::)*([A-Za-z_0-9]+)", name)
    return m.group(1) if m else name


def per_kernel_all(path):
    """{kernel: {counter: mean value per dispatch}} of a --pmc pass."""
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in agg.items()}


def library_sha256(repo):
    """sha256 of the product library in `repo` (XH_LIB_PATH when set: the
    library the profiled process loaded)."""
    path = os.environ.get("XH_LIB_PATH") or os.path.join(
        repo, "dependence_free_rl_amd", "libxylo_hip.so")
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


def main(tag, trace, fetch, write, *sq_dirs):
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = os.environ.get("PROFILE_OUT", os.path.join(here, "profiles"))
    os.makedirs(out, exist_ok=True)
    stats = glob.glob(os.path.join(trace, "**", "*kernel_stats.csv"), recursive=True)[0]
    shutil.copy(stats, os.path.join(out, "%s_kernel_stats.csv" % tag))
    dur = {r["Name"]: float(r["AverageNs"]) for r in csv.DictReader(open(stats))}
    fs, ws = per_kernel(fetch, "FETCH_SIZE"), per_kernel(write, "WRITE_SIZE")
    summary = {}
    for k in sorted(set(fs) | set(ws)):
        fb = fs.get(k, 0.0) * 1024
        wb = ws.get(k, 0.0) * 1024
        summary[short(k)] = {"kernel": k, "avg_ns": dur.get(k), "fetch_bytes_raw": fb,
                      "fetch_bytes_x2": 2 * fb, "write_bytes": wb,
                      "hbm_bytes": 2 * fb + wb, "hbm_bytes_raw_reads": fb + wb}
    # SQ / GRBM passes (MFMA utilisation): raw per-dispatch means, plus
    #   clock_ghz       = GRBM_GUI_ACTIVE / 8 XCDs / duration
    #   mfma_busy_frac  = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024
    #                     SIMDs): share of SIMD-cycles the matrix pipe was busy
    for d in sq_dirs:
        for k, cnt in per_kernel_all(d).items():
            e = summary.setdefault(short(k), {"kernel": k, "avg_ns": dur.get(k)})
            e.setdefault("sq", {}).update(cnt)
    for e in summary.values():
        sq = e.get("sq", {})
        g, ns = sq.get("GRBM_GUI_ACTIVE"), e.get("avg_ns")
        if g and ns:
            e["clock_ghz"] = g / 8.0 / ns
        if g and "SQ_VALU_MFMA_BUSY_CYCLES" in sq:
            e["mfma_busy_frac"] = sq["SQ_VALU_MFMA_BUSY_CYCLES"] / (g / 8.0 * 1024)
        # mean resident waves per SIMD (SQ_WAVE_CYCLES counts quad-cycles,
        # MI355X_MICROARCH.md) and where the waves' cycles went
        wc = sq.get("SQ_WAVE_CYCLES")
        if g and wc:
            e["occupancy"] = 4.0 * wc / (g / 8.0 * 1024)
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in sq:
                    e[c.lower() + "_frac"] = sq[c] / wc
    summary["_meta"] = {
        "tag": tag,
        "library_sha256": library_sha256(here),
        "created": datetime.datetime.now(datetime.timezone.utc).isoformat(
            timespec="seconds")}
    # PMC_META (JSON object): what the profiled run was, for lookups that
    # depend on more than the kernel's name (bench.py --env-only matches the
    # env count: its bytes per launch scale with it)
    if os.environ.get("PMC_META"):
        summary["_meta"].update(json.loads(os.environ["PMC_META"]))
    with open(os.path.join(out, "%s_pmc_summary.json" % tag), "w") as f:
        json.dump(summary, f, indent=1, sort_keys=True)
    key = os.environ.get("PMC_PRINT", "policy_train")
    print(json.dumps({k: v for k, v in summary.items() if key in k}, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
