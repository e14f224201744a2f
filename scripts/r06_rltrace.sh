#!/bin/bash
# Round 6: per-tile RL encode trace on 1 GiB runs32 with
# each tile's XCC / CU / SIMD, and the input, for scripts/trace_where.py.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06_rltrace
mkdir -p $O
TRACE_OUT=$O/trace_runs32.bin INPUT_OUT=/tmp/rl_in.bin timeout -k 10 120 scripts/ubench_rl_TRACE.bin 3 1073741824 10 > $O/ubench.log 2>&1 || { echo "trace run failed"; tail -5 $O/ubench.log; exit 1; }
cat $O/ubench.log
python3 scripts/trace_where.py $O/trace_runs32.bin /tmp/rl_in.bin > $O/where.txt 2>&1 || { echo "analysis failed"; tail -5 $O/where.txt; exit 1; }
python3 scripts/trace_stats.py $O/trace_runs32.bin > $O/stats.txt 2>&1
cat $O/where.txt
TRACE_OUT=$O/trace_runs32_b.bin timeout -k 10 120 scripts/ubench_rl_TRACE.bin 3 1073741824 10 > $O/ubench_b.log 2>&1 && python3 scripts/trace_where.py $O/trace_runs32_b.bin > $O/where_b.txt 2>&1
