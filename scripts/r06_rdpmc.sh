#!/bin/bash
# Round 6: PMC of the RL block decode on 1 GiB runs32, the round-5 kernel (base)
# against the register-rank variant (rdb_u2: bitmap words and prefixes held in
# registers, two barriers per window instead of five).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
for v in base rdb_u2; do
  bash scripts/pmc_ab.sh rl_decode runs32 scripts/ab_libs/libflrl_$v.so rd_runs32_$v > gpurun_out/rdpmc_$v.log 2>&1 || { echo "pmc $v failed"; tail -5 gpurun_out/rdpmc_$v.log; exit 1; }
  echo "== $v"; grep -A20 "rl_decode_kernel" gpurun_out/rdpmc_$v.log
done
