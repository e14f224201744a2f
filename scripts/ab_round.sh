#!/bin/bash
# this round's A/B call (GPU box)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
BASE=old EXTRA=scripts/ab_libs/libflrl_pf2w5.so,scripts/ab_libs/libflrl_pf2w4.so OPS="rl_encode:runs32,u8,upto12,longruns,zero,runs32@268435456" REPS=25 bash scripts/gpu_ab.sh || exit 1
timeout -k 10 200 python3 scripts/dbg_dec.py 1000003 131072 268435456 4096 1073741824 || exit 1
NOPMC=1 bash scripts/pmc_ab.sh fl_decode u8 scripts/ab_libs/libflrl_old.so dec_old || exit 1
NOPMC=1 bash scripts/pmc_ab.sh fl_decode u8 fl-rl-compression-mpi_amd/lib/libflrl.so dec_new || exit 1
BASE=old OPS="fl_decode:u8,lo4,u8@268435456,u8@17179869184,u8@1000003" REPS=20 bash scripts/gpu_ab.sh || exit 1
