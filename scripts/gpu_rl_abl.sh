set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 120 scripts/ubench_read.bin > gpurun_out/read.log 2>&1; cat gpurun_out/read.log | tail -3
bash scripts/rl_ablate.sh 3 2>&1 | tee gpurun_out/rl_abl.log || exit 1
timeout -k 10 600 python -u scripts/bench_stream.py --bytes 2147483648 --mem-only --sweep --reps 3 > gpurun_out/mem_sweep2.jsonl 2>gpurun_out/mem_sweep2.err || { echo "sweep failed"; tail -20 gpurun_out/mem_sweep2.err; exit 1; }
cat gpurun_out/mem_sweep2.jsonl
