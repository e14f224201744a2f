set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_rl.py tests/test_gpu_fl.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_rl.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_rl.log; exit 1; }
tail -1 gpurun_out/pytest_rl.log
bash scripts/rl_ablate.sh 3 2>&1 | tee gpurun_out/rl_abl64.log || exit 1
bash scripts/rl_ablate.sh 3 2>&1 | tee -a gpurun_out/rl_abl64.log || exit 1
