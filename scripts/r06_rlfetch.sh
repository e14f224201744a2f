#!/bin/bash
# Round 6: where the encodes' extra fetch comes
# from -- FETCH_SIZE, WRITE_SIZE and the TCC read-request split (32-byte,
# all, 128-byte "bubble", DRAM) of the shipped kernels against PMC builds
# without look-back status traffic: FLRL_RL_PMC_NOLB (RL encode, output wrong,
# so outputs are not compared) and FLRL_FL_STATIC_W=8 (FL encode, exact on u8).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
G="FETCH_SIZE;WRITE_SIZE;TCC_BUBBLE_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_DRAM_sum"
for v in "rl_encode runs32 base scripts/ab_libs/libflrl_base.so" "rl_encode runs32 nolb scripts/ab_libs/libflrl_rl_nolb.so" \
         "fl_encode u8 base scripts/ab_libs/libflrl_base.so" "fl_encode u8 static8 scripts/ab_libs/libflrl_static8.so"; do
  set -- $v
  NOPMC= PMC_GROUPS="$G" bash scripts/pmc_ab.sh $1 $2 $4 fetch_$1_$3 > gpurun_out/fetch_$1_$3.log 2>&1 || { echo "pmc $1 $3 failed"; tail -8 gpurun_out/fetch_$1_$3.log; exit 1; }
  echo "== $1 $3"; grep -A9 "${1}_.*kernel\|$1" gpurun_out/fetch_$1_$3.log | grep -A9 "kernel<" | head -10
done
