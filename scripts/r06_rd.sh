#!/bin/bash
# Round 6: RL block decode with the window's rank held in registers (per-wave
# regions, two barriers per window): RL GPU tests on the in-tree library, then
# decode call time against the round-5 build (base) for chunk-loop unrolls 1/2/4.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06_rd
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_rl.py -x -q --timeout 120 --timeout-method thread > $O/pytest_rl.log 2>&1 || { echo "rl tests failed"; tail -30 $O/pytest_rl.log; exit 1; }
tail -2 $O/pytest_rl.log
L=scripts/ab_libs/libflrl_base.so,scripts/ab_libs/libflrl_rdb_u1.so,scripts/ab_libs/libflrl_rdb_u2.so,scripts/ab_libs/libflrl_rdb_u4.so
for k in ${KINDS:-runs32 longruns zero upto16 upto24 upto64 upto200}; do
  timeout -k 10 200 python -u scripts/ab_libs.py --op rl_decode --libs $L --kind $k --reps 20 > $O/$k.log 2>&1 || { echo "fail $k"; tail -5 $O/$k.log; exit 1; }
  tail -5 $O/$k.log
done
timeout -k 10 150 python -u scripts/ab_libs.py --op rl_decode --libs $L --kind runs32 --bytes 268435456 --reps 20 > $O/n256m.log 2>&1 || { echo "fail 256m"; tail -5 $O/n256m.log; exit 1; }
tail -5 $O/n256m.log
