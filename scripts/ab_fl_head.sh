#!/bin/bash
# FL encode head tiles (FLRL_FL_HEAD): outputs against the base build over
# sizes around the head threshold, then 1 GiB / 16 GiB timing.
set -o pipefail
mkdir -p gpurun_out/ab_head
L=scripts/ab_libs/libflrl_base.so,scripts/ab_libs/libflrl_head.so,scripts/ab_libs/libflrl_head8.so
for nb in 67108864 67109253 70000001 100663296; do
  timeout -k 10 120 python -u scripts/ab_libs.py --op fl_encode --libs $L --kind u8 --bytes $nb --reps 3 > gpurun_out/ab_head/chk_$nb.log 2>&1 || { echo "fail $nb"; tail -5 gpurun_out/ab_head/chk_$nb.log; exit 1; }
  head -1 gpurun_out/ab_head/chk_$nb.log
done
for k in u8 lo4 zero lo1; do
  timeout -k 10 150 python -u scripts/ab_libs.py --op fl_encode --libs $L --kind $k --reps 30 > gpurun_out/ab_head/$k.log 2>&1 || { echo "fail $k"; tail -5 gpurun_out/ab_head/$k.log; exit 1; }
  tail -4 gpurun_out/ab_head/$k.log
done
timeout -k 10 200 python -u scripts/ab_libs.py --op fl_encode --libs $L --kind u8 --bytes 17179869184 --reps 8 > gpurun_out/ab_head/u8_16g.log 2>&1 || { echo "fail 16g"; tail -5 gpurun_out/ab_head/u8_16g.log; exit 1; }
tail -4 gpurun_out/ab_head/u8_16g.log
