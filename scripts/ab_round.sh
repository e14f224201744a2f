#!/bin/bash
# this round's A/B call (GPU box)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
BASE=old OPS="rl_decode:runs32,u8,upto12,upto32,longruns,zero,runs32@268435456" REPS=25 bash scripts/gpu_ab.sh || exit 1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_rl.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_rl.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_rl.log; exit 1; }
tail -2 gpurun_out/pytest_rl.log
bash scripts/pmc_ab.sh rl_decode runs32 fl-rl-compression-mpi_amd/lib/libflrl.so r04_dec_runs32 > gpurun_out/pmc_dec.log 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/pmc_dec.log; exit 1; }
grep -A16 "rl_decode_kernel" gpurun_out/pmc_dec.log
