#!/bin/bash
# Round 6: dense RL decode with the offsets folded in (rl_decode_dense_kernel,
# blocks of 64 K runs resolved by look-back) -- the RL GPU tests on the in-tree
# library, then the decode call against the round-5 two-kernel form (base).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06_fd
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_rl.py -x -q --timeout 120 --timeout-method thread > $O/pytest_rl.log 2>&1 || { echo "rl tests failed"; tail -30 $O/pytest_rl.log; exit 1; }
tail -2 $O/pytest_rl.log
L=${LIBS:-scripts/ab_libs/libflrl_base.so,scripts/ab_libs/libflrl_fd1.so,scripts/ab_libs/libflrl_fd_fg2.so,scripts/ab_libs/libflrl_fd_lb32.so}
for k in ${KINDS:-u8 upto2 upto4 upto8 upto12}; do
  timeout -k 10 200 python -u scripts/ab_libs.py --op rl_decode --libs $L --kind $k --reps 20 > $O/$k.log 2>&1 || { echo "fail $k"; tail -5 $O/$k.log; exit 1; }
  tail -4 $O/$k.log
done
for nb in 1000003 33554437 268435456; do
  timeout -k 10 150 python -u scripts/ab_libs.py --op rl_decode --libs $L --kind u8 --bytes $nb --reps 10 > $O/n$nb.log 2>&1 || { echo "fail n $nb"; tail -5 $O/n$nb.log; exit 1; }
  tail -4 $O/n$nb.log
done
