#!/usr/bin/env python3
"""Summarise a tools/profile.sh output directory (rocprofv3 CSVs).

Per kernel: dispatches, average duration over the last `--last` dispatches (the timed,
steady-state steps; warmup launches may be sub-batched), and per-dispatch PMC values.
HBM bytes per dispatch = WRITE_SIZE + 2 x FETCH_SIZE (KB units), the gfx950 correction of
/opt/skills/guides/MI355X_MICROARCH.md (FETCH_SIZE tallies 128-B requests at 64 B).

usage: prof_summary.py PROFILE_DIR [--last N] [--json OUT]
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


def short(name):
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"\(.*$", "", name)
    return name.replace("smcrt::", "")


def read(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def find(d, stem, kind):
    hits = glob.glob(os.path.join(d, stem, "**", f"*{kind}*.csv"), recursive=True) + \
        glob.glob(os.path.join(d, f"{stem}*.csv"))
    return hits[0] if hits else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--source", default="", help="the committed profiles/ directory these numbers are copied to")
    ap.add_argument("dir")
    ap.add_argument("--last", type=int, default=3)
    ap.add_argument("--json")
    ap.add_argument("--traffic", help="write profiles/transport_traffic.json-style file here")
    ap.add_argument("--batch", type=int, default=4_000_000)
    ap.add_argument("--grid", type=int, default=128)
    ap.add_argument("--workload", default="m1")
    a = ap.parse_args()
    out = {}
    tr = os.path.join(a.dir, "kernel_trace.csv")  # (a copied summary directory)
    if not os.path.exists(tr):
        tr = find(a.dir, "trace", "kernel_trace")
    disp = defaultdict(list)
    for r in (read(tr) if tr else []):
        k = short(r["Kernel_Name"])
        disp[k].append((int(r["Dispatch_Id"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6,
                        int(r["VGPR_Count"]), int(r["SGPR_Count"])))
    for k, v in disp.items():
        v.sort()
        tail = v[-a.last:]
        out[k] = {"dispatches": len(v), "avg_ms_last": sum(x[1] for x in tail) / len(tail),
                  "total_ms": sum(x[1] for x in v)}
    for stem in ("pmc_sq", "pmc_fetch", "pmc_write", "pmc_tcc", "pmc_valu"):
        p = find(a.dir, stem, "counter_collection") or (os.path.join(a.dir, stem + ".csv")
                                                         if os.path.exists(os.path.join(a.dir, stem + ".csv")) else None)
        if not p:
            continue
        per = defaultdict(lambda: defaultdict(list))
        for r in read(p):
            per[short(r["Kernel_Name"])][r["Counter_Name"]].append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
        for k, cs in per.items():
            if k not in out:
                if tr:
                    continue
                out[k] = {"dispatches": 0, "avg_ms_last": 0.0, "total_ms": 0.0}  # (a PMC-only directory)
            for c, v in cs.items():
                v.sort()
                tail = v[-a.last:]
                out[k][c] = sum(x[1] for x in tail) / len(tail)
    for k, d in out.items():
        if "WRITE_SIZE" in d or "FETCH_SIZE" in d:
            d["hbm_bytes_per_dispatch"] = 1024.0 * (d.get("WRITE_SIZE", 0.0) + 2.0 * d.get("FETCH_SIZE", 0.0))
            d["hbm_GBps"] = d["hbm_bytes_per_dispatch"] / (d["avg_ms_last"] * 1e-3) / 1e9 if d["avg_ms_last"] else 0.0
    tot = sum(d["avg_ms_last"] for k, d in out.items() if "rocclr" not in k and "elementwise" not in k) or 1.0
    for k, d in sorted(out.items(), key=lambda kv: -kv[1]["avg_ms_last"]):
        if "rocclr" in k or "elementwise" in k:
            continue
        extra = "".join(f" {c}={d[c]:.4g}" for c in sorted(d) if c.isupper() or c.startswith("SQ") or c.startswith("TCC"))
        hb = f" hbm={d['hbm_bytes_per_dispatch']/1e9:.3f}GB ({d['hbm_GBps']:.0f} GB/s)" if "hbm_GBps" in d else ""
        print(f"{k:28s} n={d['dispatches']:3d} avg={d['avg_ms_last']:8.3f} ms ({100*d['avg_ms_last']/tot:5.1f}%)"
              f"{hb}{extra}")
    if a.traffic:
        k = next((k for k in out if k.startswith(("transport_kernel", "ws_kernel")) and
                  "hbm_bytes_per_dispatch" in out[k]), None)
        if k:
            # the whole step: the transport kernel plus the deposit-fold kernels that follow each
            # of its launches (same dispatch count), per launch
            step = {kk: out[kk]["hbm_bytes_per_dispatch"] for kk in out
                    if (kk == k or kk.startswith(("bin_", "bk_", "dda_", "fold_")))
                    and "hbm_bytes_per_dispatch" in out[kk]}
            classes = {c: out[k][c] for c in out[k] if c.startswith("SQ_INSTS_VALU_")}
            with open(a.traffic, "w") as f:
                json.dump({"workload": a.workload, "batch": a.batch, "grid": a.grid, "kernel": k,
                           "hbm_bytes_per_launch": out[k]["hbm_bytes_per_dispatch"],
                           "step_hbm_bytes_per_launch": sum(step.values()),
                           "hbm_bytes_per_launch_by_kernel": step,
                           "valu_insts_per_launch": out[k].get("SQ_INSTS_VALU"),
                           "salu_insts_per_launch": out[k].get("SQ_INSTS_SALU"),
                           "valu_classes": classes,
                           "avg_ms": out[k]["avg_ms_last"], "source": a.source or os.path.relpath(a.dir)}, f, indent=1)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
