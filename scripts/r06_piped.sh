#!/bin/bash
# Round 6: dense RL decode with the offsets folded in (rl_decode_piped_kernel,
# the in-tree build) against the two-kernel form (LIBS' first build); decode
# call time, outputs compared with the first build's.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06_piped
mkdir -p $O
L=${LIBS:-scripts/ab_libs/libflrl_base.so,fl-rl-compression-mpi_amd/lib/libflrl.so}
for k in ${KINDS:-u8 upto2 upto4 upto8 upto12 runs32}; do
  timeout -k 10 200 python -u scripts/ab_libs.py --op rl_decode --libs $L --kind $k --reps ${REPS:-20} > $O/$k.log 2>&1 || { echo "fail $k"; tail -5 $O/$k.log; exit 1; }
  tail -3 $O/$k.log
done
for nb in ${SIZES:-1048576 104857600 4294967296}; do
  timeout -k 10 200 python -u scripts/ab_libs.py --op rl_decode --libs $L --kind u8 --bytes $nb --reps 15 > $O/n$nb.log 2>&1 || { echo "fail n $nb"; tail -5 $O/n$nb.log; exit 1; }
  tail -3 $O/n$nb.log
done
