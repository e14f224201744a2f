#!/bin/bash
# this round's A/B call (GPU box)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fl.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_fl.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_fl.log; exit 1; }
tail -2 gpurun_out/pytest_fl.log
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_rl.py tests/test_gpu_stream.py tests/test_gpu_shard.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_rest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_rest.log; exit 1; }
tail -2 gpurun_out/pytest_rest.log
BASE=old OPS="fl_decode:u8,lo4,u8@268435456,u8@17179869184" REPS=20 bash scripts/gpu_ab.sh || exit 1
bash scripts/pmc_ab.sh rl_encode runs32 fl-rl-compression-mpi_amd/lib/libflrl.so r04_enc_runs32_new > gpurun_out/pmc_new.log 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/pmc_new.log; exit 1; }
grep -A16 "rl_encode_wave" gpurun_out/pmc_new.log
