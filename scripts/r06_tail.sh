#!/bin/bash
# Round 6: RL encode with shorter tail tiles (FLRL_RL_TAIL_TILES x FLRL_RL_TAIL_BYTES
# at the end of the input) against the shipped 128 KiB tiles; encode call time.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06_tail
mkdir -p $O
L=${LIBS:-scripts/ab_libs/libflrl_tail0.so,scripts/ab_libs/libflrl_tail32k_512.so,scripts/ab_libs/libflrl_tail32k_1280.so,scripts/ab_libs/libflrl_tail64k_1280.so,scripts/ab_libs/libflrl_tail64k_2560.so}
for k in ${KINDS:-runs32 longruns zero u8 upto12}; do
  timeout -k 10 200 python -u scripts/ab_libs.py --op rl_encode --libs $L --kind $k --reps 25 > $O/$k.log 2>&1 || { echo "fail $k"; tail -5 $O/$k.log; exit 1; }
  tail -6 $O/$k.log
done
for nb in 104857600 268435456 4294967296; do
  timeout -k 10 200 python -u scripts/ab_libs.py --op rl_encode --libs $L --kind runs32 --bytes $nb --reps 15 > $O/n$nb.log 2>&1 || { echo "fail n $nb"; tail -5 $O/n$nb.log; exit 1; }
  tail -6 $O/n$nb.log
done
