#!/usr/bin/env python3
"""Summarise a scripts/profile.sh run into profiles/<tag>_*.

Reads gpurun_out/prof/<tag>/{trace,fetch,write}/*.csv and writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --stats summary (verbatim)
  profiles/<tag>_summary.json       per-kernel avg duration, HBM bytes/launch
  profiles/traffic_<kind>_<bytes>.json  read by bench.py for roofline.traffic of that workload
HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are KiB;
on gfx950 FETCH_SIZE reports half the bytes of a wide (16 B/lane) coalesced
streaming read, so it is doubled; WRITE_SIZE is exact for 16-B stores.
Usage: summarize_profile.py <tag> [--bytes N --kind u8]
"""
import argparse
import csv
import json
import os
import re
import shutil
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KMAP = {"fl_encode_kernel": "fl_encode", "fl_decode_kernel": "fl_decode",
        "fl_offsets_kernel": "fl_offsets", "rl_encode_wave_kernel": "rl_encode",
        "rl_encode_scan_kernel": "rl_encode_scan", "rl_encode_state_kernel": "rl_encode_state",
        "rl_encode_emit_kernel": "rl_encode_emit",
        "rl_decode_kernel": "rl_decode", "rl_decode_wave_kernel": "rl_decode_wave", "rl_offsets_kernel": "rl_offsets",
        "gen_kernel": "gen", "zero_kernel": "zero"}


def short(name: str) -> str:
    for k, v in KMAP.items():
        if k in name:
            return v
    return re.sub(r"\(.*", "", name)[:60]


def pmc(path, counter):
    out = {}
    if not os.path.exists(path):
        return out
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        out.setdefault(short(r["Kernel_Name"]), []).append(float(r["Counter_Value"]) * 1024)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--bytes", type=int, default=1 << 30)
    ap.add_argument("--kind", default="u8")
    a = ap.parse_args()
    src = os.path.join(ROOT, "gpurun_out", "prof", a.tag)
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(dst, f"{a.tag}_kernel_stats.csv"))
    durs = {}
    for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_trace.csv"))):
        d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        durs.setdefault(short(r["Kernel_Name"]), []).append(d)
    fetch = pmc(os.path.join(src, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = pmc(os.path.join(src, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    kernels = {}
    for k, v in durs.items():
        e = {"calls": len(v), "avg_ns": round(statistics.mean(v), 1),
             "median_ns": statistics.median(v), "min_ns": min(v), "max_ns": max(v)}
        if k in fetch and k in write:
            f = statistics.median(fetch[k]) * 2  # gfx950 FETCH_SIZE = half of streamed bytes
            w = statistics.median(write[k])
            e.update({"fetch_bytes_raw": statistics.median(fetch[k]), "fetch_bytes_corrected": f,
                      "write_bytes": w, "hbm_bytes_per_launch": int(f + w)})
        kernels[k] = e
    summary = {"tag": a.tag, "bytes": a.bytes, "kind": a.kind,
               "method": "rocprofv3 --kernel-trace --stats; --pmc FETCH_SIZE and --pmc WRITE_SIZE "
                         "in separate passes; FETCH_SIZE x2 (gfx950 wide-read correction)",
               "kernels": kernels}
    with open(os.path.join(dst, f"{a.tag}_summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    with open(os.path.join(dst, f"traffic_{a.kind}_{a.bytes}.json"), "w") as f:
        json.dump(summary, f, indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
