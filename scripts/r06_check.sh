#!/bin/bash
# Round 6: smoke + every GPU test + default bench line on the current tree, then
# the N = 1 line through the RCCL exchange (--force-scan, configs4 section).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_check.sh || exit 1
cp gpurun_out/bench.log gpurun_out/bench_default.log
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr=127.0.0.1 --master-port=29533 \
    bench.py --gpus 1 --force-scan --no-rl --no-configs3 --no-north-star > gpurun_out/bench_forcescan.log 2>&1 || { echo "forcescan bench failed"; tail -20 gpurun_out/bench_forcescan.log; exit 1; }
tail -1 gpurun_out/bench_forcescan.log | cut -c1-600
