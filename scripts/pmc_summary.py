#!/usr/bin/env python3
"""Per-kernel means of a scripts/pmc_ab.sh run: durations from the kernel
trace, counters per dispatch (summed over XCDs/instances) from the --pmc passes."""
import csv
import glob
import os
import sys
from collections import defaultdict

out = sys.argv[1]
only = sys.argv[2] if len(sys.argv) > 2 else ""  # keep kernels whose name contains this
dur = defaultdict(list)
for f in glob.glob(os.path.join(out, "trace", "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        dur[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
cnt = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
for f in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        cnt[r["Kernel_Name"]][r["Counter_Name"]][r["Dispatch_Id"] + f] += float(r["Counter_Value"])
for k in sorted(set(dur) | set(cnt)):
    if only not in k:
        continue
    short = k.split("(")[0][-60:]
    d = dur.get(k, [])
    print(f"{short}: calls {len(d)} mean {sum(d) / len(d) / 1e3:.1f} us" if d else f"{short}:")
    for c, per in sorted(cnt.get(k, {}).items()):
        v = list(per.values())
        print(f"    {c:24s} {sum(v) / len(v):16.4g}")
