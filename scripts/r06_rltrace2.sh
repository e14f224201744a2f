#!/bin/bash
# Round 6: RL encode per-tile traces, 64-tile (shipped) vs 128-tile look-back
# windows (FLRL_RL_LOOKG=2), 1 GiB runs32, for scripts/trace_stats.py.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06_rltrace2
mkdir -p $O
for v in "g1 scripts/ubench_rl_TRACE.bin" "g2 scripts/ubench_rl_TRACE_g2.bin"; do
  set -- $v
  TRACE_OUT=$O/trace_$1.bin timeout -k 10 120 $2 3 1073741824 10 > $O/ubench_$1.log 2>&1 || { echo "trace $1 failed"; tail -5 $O/ubench_$1.log; exit 1; }
  head -1 $O/ubench_$1.log
  python3 scripts/trace_stats.py $O/trace_$1.bin > $O/stats_$1.txt 2>&1
  head -12 $O/stats_$1.txt
done
