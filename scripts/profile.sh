#!/bin/bash
# rocprofv3 evidence for bench.py (run on the GPU box via gpurun):
#   1. --kernel-trace --stats        per-kernel durations (must agree with bench.py's HIP events)
#   2. --pmc FETCH_SIZE              HBM read bytes per dispatch  (own pass)
#   3. --pmc WRITE_SIZE              HBM write bytes per dispatch (own pass)
# Outputs land in gpurun_out/prof/<tag>/; scripts/summarize_profile.py turns them
# into profiles/<tag>_*.{csv,json}. Usage: bash scripts/profile.sh <tag> [bench args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-r01}
shift
BENCH_ARGS=("$@")
# the 16 GiB north-star launches would mix into the 1 GiB kernel averages: profile them separately
[ ${#BENCH_ARGS[@]} -eq 0 ] && BENCH_ARGS=(--no-north-star --no-rl-dense --no-configs3)
OUT=gpurun_out/prof/$TAG
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run \
    -- python3 bench.py --steps 20 --warmup 5 --cpu-sample 0 "${BENCH_ARGS[@]}" > "$OUT/trace.log" 2>&1 || { echo "trace pass failed"; tail -20 "$OUT/trace.log"; exit 1; }
echo "trace pass ok"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run \
    -- python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 "${BENCH_ARGS[@]}" > "$OUT/fetch.log" 2>&1 || { echo "fetch pass failed"; tail -20 "$OUT/fetch.log"; exit 1; }
echo "fetch pass ok"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run \
    -- python3 bench.py --steps 3 --warmup 1 --cpu-sample 0 "${BENCH_ARGS[@]}" > "$OUT/write.log" 2>&1 || { echo "write pass failed"; tail -20 "$OUT/write.log"; exit 1; }
echo "write pass ok"
find "$OUT" -name "*.csv" | head -20
