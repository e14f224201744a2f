#!/bin/bash
# Round-4 (session 2): FL decode GPU tests on the working-tree library, then the
# RL encode runs32 per-tile trace (occupancy over the launch).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fl.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_fl.log 2>&1 || { echo "fl tests failed"; tail -30 gpurun_out/pytest_fl.log; exit 1; }
tail -2 gpurun_out/pytest_fl.log
timeout -k 10 120 ./scripts/ubench_rl_TRACE.bin 3 1073741824 5 > gpurun_out/ub_trace.log 2>&1 || { echo "trace failed"; tail -5 gpurun_out/ub_trace.log; exit 1; }
tail -3 gpurun_out/ub_trace.log
python3 scripts/trace_stats.py gpurun_out/rl_trace.bin > gpurun_out/trace_stats.log 2>&1
cat gpurun_out/trace_stats.log
