#!/bin/bash
# FL encode/decode time against size (u8, device-resident, HIP events in
# scripts/ubench_fl_plain.bin), then a rocprofv3 kernel trace at two sizes:
# the intercept of time(n) is the per-launch fixed cost. GPU box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/fl_sweep
for b in 134217728 268435456 536870912 1073741824 2147483648 4294967296 8589934592; do
  timeout -k 10 120 ./scripts/ubench_fl_plain.bin ${KIND:-0} $b 20 || exit 1
done
for b in 1073741824 4294967296; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fl_sweep/t_$b -o run -- ./scripts/ubench_fl_plain.bin ${KIND:-0} $b 20 > gpurun_out/fl_sweep/t_$b.log 2>&1 || exit 1
done
find gpurun_out/fl_sweep -name "*kernel_stats.csv" | while read f; do echo "== $f"; cut -d, -f1-5 "$f" | head -8; done
