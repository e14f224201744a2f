#!/bin/bash
# Round-4 first look (GPU box): RL encode runs32 timing, per-tile trace and the
# SQ counters of the current kernel (the "before" PMC under profiles/r04_*).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/ubench_rl_plain.bin 3 1073741824 20 > gpurun_out/ub_plain.log 2>&1 || { echo "plain failed"; tail -5 gpurun_out/ub_plain.log; exit 1; }
cat gpurun_out/ub_plain.log
timeout -k 10 120 ./scripts/ubench_rl_TRACE.bin 3 1073741824 5 > gpurun_out/ub_trace.log 2>&1 || { echo "trace failed"; tail -5 gpurun_out/ub_trace.log; exit 1; }
python3 scripts/trace_stats.py gpurun_out/rl_trace.bin > gpurun_out/trace_stats.log 2>&1
cat gpurun_out/trace_stats.log
bash scripts/pmc_ab.sh rl_encode runs32 fl-rl-compression-mpi_amd/lib/libflrl.so r04_rl_encode_runs32_before > gpurun_out/pmc_enc.log 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/pmc_enc.log; exit 1; }
cat gpurun_out/pmc_enc.log
