#!/bin/bash
# Round-5 RL encode check on the GPU box: probe the persistent encode on dense
# kinds against the previous form, the RL GPU tests, then an A/B per kind.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 python3 scripts/lag_probe.py --kinds u8,longruns,zero \
    --libs scripts/ab_libs/libflrl_old.so,scripts/ab_libs/libflrl_guard.so 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_rl.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r05_lag_rltest.log 2>&1
rc=$?
tail -3 gpurun_out/r05_lag_rltest.log
[ $rc -eq 0 ] || exit $rc
OPS="${OPS:-rl_encode:runs32,upto12,upto24,longruns,zero,u8,upto4,runs32@268435456}" BASE=old REPS=${REPS:-20} \
    timeout -k 10 250 bash scripts/gpu_ab.sh 2>&1 | grep -v amdgpu.ids
