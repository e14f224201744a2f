#!/bin/bash
# Round 6: RL decode offsets pre-pass with 32 count vectors per lane per step
# (one load round for 1 GiB runs32) against the shipped 16; decode call time.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06_ro
mkdir -p $O
L=scripts/ab_libs/libflrl_base.so,scripts/ab_libs/libflrl_ro32.so
for k in runs32 u8 upto4 upto16 longruns zero; do
  timeout -k 10 200 python -u scripts/ab_libs.py --op rl_decode --libs $L --kind $k --reps 30 > $O/$k.log 2>&1 || { echo "fail $k"; tail -5 $O/$k.log; exit 1; }
  tail -3 $O/$k.log
done
for nb in 268435456 4294967296; do
  timeout -k 10 200 python -u scripts/ab_libs.py --op rl_decode --libs $L --kind runs32 --bytes $nb --reps 20 > $O/n$nb.log 2>&1 || { echo "fail $nb"; tail -5 $O/n$nb.log; exit 1; }
  tail -3 $O/n$nb.log
done
