#!/bin/bash
# Interleaved timing of prebuilt RL ubench binaries over input kinds (GPU box).
# Usage: bash scripts/rl_ab_bins.sh "binA binB ..." "kinds"
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
BINS=${1:-"scripts/ubench_rl_lb128.bin scripts/ubench_rl_lb64.bin"}
KINDS=${2:-"3 4 2 0 1 104 108 112 124"}
for k in $KINDS; do
  for rep in 1 2; do
    for b in $BINS; do
      echo -n "$(basename $b) kind $k: "
      timeout -k 10 60 $b $k 1073741824 15 | tr '\n' ' ' | sed 's/rl_encode kind [0-9]* n [0-9]* //' || exit 1
      echo
    done
  done
done
