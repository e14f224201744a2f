#!/bin/bash
# A/B of the working-tree library against a baseline build (scripts/ab_libs/libflrl_$BASE.so)
# over ops and input kinds, then the GPU tests selected by $PYTEST_K (GPU box).
# Usage: BASE=old OPS="rl_decode:runs32,u8 fl_decode:u8" bash scripts/gpu_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
LIBS="scripts/ab_libs/libflrl_${BASE:-old}.so,fl-rl-compression-mpi_amd/lib/libflrl.so${EXTRA:+,$EXTRA}"
for spec in $OPS; do
  op=${spec%%:*}; kinds=${spec#*:}
  for k in ${kinds//,/ }; do
    b=""; case $k in *@*) b="--bytes ${k#*@}"; k=${k%@*};; esac
    echo "== $op $k $b"
    timeout -k 10 120 python3 scripts/ab_libs.py --op "$op" --libs "$LIBS" --kind "$k" $b --reps ${REPS:-20} ${DIRTY:+--dirty $DIRTY} ${NOCHECK:+--nocheck} ${CLEAN:+--clean $CLEAN} || exit 1
  done
done
if [ -n "$PYTEST_K" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$PYTEST_K" > gpurun_out/pytest_ab.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_ab.log; exit 1; }
  tail -2 gpurun_out/pytest_ab.log
fi
