#!/bin/bash
# Round 6 default-workload evidence: the bench line (saved), then rocprofv3
# kernel trace + FETCH_SIZE + WRITE_SIZE passes of the same command (tag r06).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/r06_bench_default.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r06_bench_default.log; exit 1; }
tail -1 gpurun_out/r06_bench_default.log | cut -c1-400
bash scripts/profile.sh r06 || exit 1
python3 scripts/summarize_profile.py r06 > gpurun_out/summ_r06.log 2>&1 || { tail -5 gpurun_out/summ_r06.log; exit 1; }
