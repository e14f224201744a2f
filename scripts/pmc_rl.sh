#!/bin/bash
# SQ instruction/cycle counters for the RL encode (scripts/ubench_rl.bin), one
# rocprofv3 --pmc pass per counter group. Run on the GPU box via gpurun.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc_rl}
mkdir -p "$OUT"
BIN=${1:-./scripts/ubench_rl.bin}
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/trace" -o run -- "$BIN" 3 1073741824 3 > "$OUT/trace.log" 2>&1 || { echo "trace pass failed"; tail -5 "$OUT/trace.log"; }
i=0
for grp in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_INSTS_BRANCH" "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD"; do
    i=$((i+1))
    timeout -k 10 200 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- "$BIN" 3 1073741824 3 > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; }
done
find "$OUT" -name "*counter_collection.csv"
