#!/bin/bash
# this round's A/B call (GPU box)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
BASE=old EXTRA=scripts/ab_libs/libflrl_pf2.so OPS="rl_encode:runs32,u8,upto12,upto4,longruns,zero,runs32@268435456" REPS=25 bash scripts/gpu_ab.sh || exit 1
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_rl.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_rl.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_rl.log; exit 1; }
tail -2 gpurun_out/pytest_rl.log
