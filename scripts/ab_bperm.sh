#!/bin/bash
# RL decode with ds_bpermute chunk values (FLRL_RD_BPERM): the RL GPU tests on
# the in-tree library, then outputs and timing against the previous build.
set -o pipefail
mkdir -p gpurun_out/ab_bperm
timeout -k 10 600 python -u -m pytest tests/test_gpu_rl.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_bperm/pytest_rl.log 2>&1 || { echo "rl tests failed"; tail -30 gpurun_out/ab_bperm/pytest_rl.log; exit 1; }
tail -2 gpurun_out/ab_bperm/pytest_rl.log
L=scripts/ab_libs/libflrl_base.so,fl-rl-compression-mpi_amd/lib/libflrl.so
for k in runs32 longruns zero upto16 upto24 upto64 upto200 u8 upto4; do
  timeout -k 10 150 python -u scripts/ab_libs.py --op rl_decode --libs $L --kind $k --reps 30 > gpurun_out/ab_bperm/$k.log 2>&1 || { echo "fail $k"; tail -5 gpurun_out/ab_bperm/$k.log; exit 1; }
  tail -3 gpurun_out/ab_bperm/$k.log
done
for nb in 1000003 33554437 268435456; do
  timeout -k 10 150 python -u scripts/ab_libs.py --op rl_decode --libs $L --kind runs32 --bytes $nb --reps 5 > gpurun_out/ab_bperm/n$nb.log 2>&1 || { echo "fail n $nb"; tail -5 gpurun_out/ab_bperm/n$nb.log; exit 1; }
  head -1 gpurun_out/ab_bperm/n$nb.log
done
