#!/bin/bash
# A/B of scripts/ab_libs/libflrl_{base,$1}.so (scripts/ab_libs.py) over a list of
# op:kind pairs, one process per pair: bash scripts/ab_quick.sh VARIANT op:kind ...
set -o pipefail
V=$1; shift
mkdir -p gpurun_out/ab_quick
L=scripts/ab_libs/libflrl_base.so,scripts/ab_libs/libflrl_$V.so
for ok in "$@"; do
  op=${ok%%:*}; k=${ok#*:}
  timeout -k 10 150 python -u scripts/ab_libs.py --op $op --libs $L --kind $k --reps 15 > gpurun_out/ab_quick/$V-$op-$k.log 2>&1 || { echo "fail $op $k"; tail -5 gpurun_out/ab_quick/$V-$op-$k.log; exit 1; }
  tail -3 gpurun_out/ab_quick/$V-$op-$k.log
done
