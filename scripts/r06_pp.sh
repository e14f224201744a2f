#!/bin/bash
# Round 6: dense RL encode emission (piece_part) variants against the shipped
# build; encode call time, outputs compared with the first build's.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06_pp
mkdir -p $O
L=${LIBS:-scripts/ab_libs/libflrl_base.so,scripts/ab_libs/libflrl_pp1.so}
for k in ${KINDS:-u8 upto2 upto4 upto8 runs32 longruns zero}; do
  timeout -k 10 200 python -u scripts/ab_libs.py --op rl_encode --libs $L --kind $k --reps ${REPS:-20} > $O/$k.log 2>&1 || { echo "fail $k"; tail -5 $O/$k.log; exit 1; }
  tail -4 $O/$k.log
done
