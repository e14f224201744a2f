set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_fl.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
FLRL_HOST_DIRECT=1 timeout -k 10 240 python -u -m pytest tests/test_gpu_fl.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_direct.log 2>&1 || { echo "pytest direct failed"; tail -40 gpurun_out/pytest_direct.log; exit 1; }
tail -1 gpurun_out/pytest_direct.log
timeout -k 10 600 python -u scripts/bench_stream.py --bytes 2147483648 --mem-only --sweep --reps 3 > gpurun_out/mem_sweep.jsonl 2>gpurun_out/mem_sweep.err || { echo "sweep failed"; tail -20 gpurun_out/mem_sweep.err; exit 1; }
cat gpurun_out/mem_sweep.jsonl
