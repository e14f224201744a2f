#!/bin/bash
# Kernel trace + SQ counters (one rocprofv3 pass per group) of one device call
# timed by scripts/ab_libs.py, then a per-kernel summary (GPU box via gpurun).
# Usage: bash scripts/pmc_ab.sh <op> <kind> [lib] [tag]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OP=$1; KIND=$2; LIB=${3:-fl-rl-compression-mpi_amd/lib/libflrl.so}; TAG=${4:-$OP_$KIND}
OUT=gpurun_out/pmc_ab/$TAG
rm -rf "$OUT"; mkdir -p "$OUT"
CMD=(python3 scripts/ab_libs.py --op "$OP" --libs "$LIB" --kind "$KIND" --reps 4 ${BYTES:+--bytes $BYTES})
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- "${CMD[@]}" > "$OUT/trace.log" 2>&1 || [ -n "$ALLOWFAIL" ] || { echo "trace failed"; tail -5 "$OUT/trace.log"; exit 1; }
[ -n "$NOPMC" ] && { python3 scripts/pmc_summary.py "$OUT"; exit 0; }
i=0
# PMC_GROUPS (';'-separated passes) overrides the default SQ groups
GROUPS_DEFAULT="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD;SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH"
IFS=';' read -ra GRPS <<< "${PMC_GROUPS:-$GROUPS_DEFAULT}"
for grp in "${GRPS[@]}"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- "${CMD[@]}" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; exit 1; }
done
python3 scripts/pmc_summary.py "$OUT"
