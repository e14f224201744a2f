#!/bin/bash
# Round-5 GPU batch: the whole GPU suite, the default bench line (with the
# configs[3] section), an FL lo4 per-tile encode trace, and the rocprofv3
# summaries (trace + FETCH/WRITE passes) of the 1 GiB default and of the
# 16 GiB lo4 workload (BASELINE configs[3]). Every step has its own time
# limit; the script stops at the first failure.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
      > gpurun_out/r05_pytest_gpu.log 2>&1
  rc=$?; tail -3 gpurun_out/r05_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python3 bench.py > gpurun_out/r05_bench.log 2>&1 || { tail -20 gpurun_out/r05_bench.log; exit 1; }
grep '^{"metric"' gpurun_out/r05_bench.log | tail -1 > gpurun_out/r05_bench_line.json
timeout -k 10 120 scripts/ubench_fl_TRACE.bin 1 1073741824 5 && python3 scripts/fl_trace_stats.py gpurun_out/fl_trace.bin || exit 1
bash scripts/profile.sh r05 || exit 1
bash scripts/profile.sh r05_lo4 --kind lo4 --bytes 17179869184 --no-north-star --no-rl --no-configs3 || exit 1
