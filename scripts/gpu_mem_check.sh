set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u scripts/bench_stream.py --bytes 2147483648 --mem-only --reps 3 > gpurun_out/mem_rates.json 2>gpurun_out/mem_rates.err || { echo "mem failed"; tail -20 gpurun_out/mem_rates.err; exit 1; }
cat gpurun_out/mem_rates.json
