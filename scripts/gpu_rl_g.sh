set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for rep in 1 2; do for g in 1 2 4 8; do echo -n "G=$g: "; timeout -k 10 60 scripts/ubench_rl_g$g.bin 3 1073741824 20 | head -2 | tr '\n' ' '; echo; done; done 2>&1 | tee gpurun_out/rl_g.log
timeout -k 10 900 python -u scripts/bench_stream.py --bytes 2147483648 --mem-only --sweep --reps 3 > gpurun_out/mem_sweep2.jsonl 2>gpurun_out/mem_sweep2.err || { echo "sweep failed"; tail -20 gpurun_out/mem_sweep2.err; exit 1; }
cat gpurun_out/mem_sweep2.jsonl
