#!/bin/bash
# The bench's RL section with each library build in turn (GPU box): copies
# scripts/ab_libs/libflrl_<v>.so over the in-tree library, runs bench.py
# without the CPU baseline, north star and configs4 sections, prints the RL
# kernel times, and restores the in-tree library.
# Usage: VARIANTS="base both" REPEAT=2 bash scripts/bench_libs.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
LIB=fl-rl-compression-mpi_amd/lib/libflrl.so
cp "$LIB" gpurun_out/libflrl.orig.so
for r in $(seq 1 "${REPEAT:-1}"); do
  for v in $VARIANTS; do
    cp "scripts/ab_libs/libflrl_$v.so" "$LIB"
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-sample 0 --no-north-star --no-configs4 > "gpurun_out/bench_$v.log" 2>&1 || { cp gpurun_out/libflrl.orig.so "$LIB"; echo "bench $v failed"; tail -5 "gpurun_out/bench_$v.log"; exit 1; }
    python3 - "$v" "gpurun_out/bench_$v.log" <<'PY'
import json, sys
line = [l for l in open(sys.argv[2]) if l.startswith('{"metric"')][-1]
b = json.loads(line); r = b["rl"]; d = r.get("dense_u8", {})
print(f"{sys.argv[1]:8s} fl_enc {b['kernels']['fl_encode']['ms']:.4f} fl_dec {b['kernels']['fl_decode']['ms']:.4f} "
      f"rl_enc {r['rl_encode']['ms']:.4f} rl_dec {r['rl_decode']['ms']:.4f} call {r['rl_decode']['call_ms']:.4f} "
      f"dense_dec {d.get('rl_decode', {}).get('ms', 0):.4f} dense_enc {d.get('rl_encode', {}).get('ms', 0):.4f}")
PY
  done
done
cp gpurun_out/libflrl.orig.so "$LIB"
