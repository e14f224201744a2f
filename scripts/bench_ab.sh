#!/bin/bash
# The default bench with the working-tree library and with variant builds
# (scripts/ab_libs/libflrl_<name>.so swapped in), alternating, on one box.
# Usage: VARIANTS="p1" ROUNDS=2 bash scripts/bench_ab.sh [bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
LIB=fl-rl-compression-mpi_amd/lib/libflrl.so
cp "$LIB" gpurun_out/libflrl_tree.so || exit 1
for r in $(seq ${ROUNDS:-2}); do
  for v in tree $VARIANTS; do
    if [ "$v" = tree ]; then cp gpurun_out/libflrl_tree.so "$LIB"; else cp "scripts/ab_libs/libflrl_$v.so" "$LIB"; fi
    timeout -k 10 300 python3 bench.py --no-north-star --cpu-sample 0 "$@" > gpurun_out/bench_$v.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/bench_$v.log; cp gpurun_out/libflrl_tree.so "$LIB"; exit 1; }
    python3 -c "
import json,sys
b=json.loads(open('gpurun_out/bench_$v.log').read().strip().splitlines()[-1])
r=b['rl']; d=r.get('dense_u8',{})
print('$v', 'fl_enc', b['kernels']['fl_encode']['ms'], 'fl_dec', b['kernels']['fl_decode']['ms'], 'rl_enc', r['rl_encode']['ms'], r['rl_encode']['call_ms'], 'rl_dec', r['rl_decode']['ms'], r['rl_decode']['call_ms'], 'u8 enc', d.get('rl_encode',{}).get('call_ms'), 'u8 dec', d.get('rl_decode',{}).get('call_ms'))
"
  done
done
cp gpurun_out/libflrl_tree.so "$LIB"
