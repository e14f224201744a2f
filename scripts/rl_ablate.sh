#!/bin/bash
# RL encode timing ablations (FLRL_RL_ABL bits, flrl_rl.hip) on the GPU box.
# Usage: bash scripts/rl_ablate.sh [kind=3] -- builds one ubench per variant first.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
KIND=${1:-3}
for a in 0 1 2 4 6 7 15; do
  [ -x scripts/ubench_rl_abl$a.bin ] || { echo "missing scripts/ubench_rl_abl$a.bin"; exit 1; }
done
for a in 0 1 2 4 6 7 15; do
  echo -n "ABL=$a: "; NO_DECODE=1 timeout -k 10 60 scripts/ubench_rl_abl$a.bin $KIND 1073741824 20 || exit 1
done
