#!/bin/bash
# this round's A/B call (GPU box)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fl.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_fl.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_fl.log; exit 1; }
tail -2 gpurun_out/pytest_fl.log
BASE=old OPS="fl_decode:u8,lo4,u8@268435456,u8@17179869184" REPS=20 bash scripts/gpu_ab.sh || exit 1
BASE=old EXTRA=scripts/ab_libs/libflrl_pf2.so OPS="rl_encode:runs32,u8,upto12,upto4,longruns,zero,runs32@268435456" REPS=25 bash scripts/gpu_ab.sh || exit 1
NOPMC=1 bash scripts/pmc_ab.sh fl_decode u8 fl-rl-compression-mpi_amd/lib/libflrl.so dec_pre || exit 1
