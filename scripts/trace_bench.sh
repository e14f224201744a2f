#!/bin/bash
# rocprofv3 kernel trace of the default bench (no PMC), per-kernel means.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/trace_bench/${1:-t}
rm -rf "$OUT"; mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT" -o run -- python3 bench.py --no-north-star --no-rl-dense --cpu-sample 0 --steps 10 --warmup 2 > "$OUT/bench.log" 2>&1 || { echo "trace failed"; tail -5 "$OUT/bench.log"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys, statistics
from collections import defaultdict
d = defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        d[r["Kernel_Name"].split("(")[0][-45:]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items()):
    if "flrl" in k:
        print(f"{k:45s} n={len(v):3d} median {statistics.median(v):9.1f} us")
PY
