#!/bin/bash
# Round 6, first GPU call: smoke + GPU tests + default bench on the trimmed RL
# sources, then the north-star workload (16 GiB u8 FL encode/decode) profiled on
# HEAD: rocprofv3 kernel trace + FETCH_SIZE + WRITE_SIZE passes (tag r06_16g_u8).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_check.sh || exit 1
bash scripts/profile.sh r06_16g_u8 --bytes 17179869184 --no-north-star --no-rl --no-rl-dense --no-configs3 || exit 1
python3 scripts/summarize_profile.py r06_16g_u8 --bytes 17179869184 --kind u8 > gpurun_out/summ16.log 2>&1 || { tail -5 gpurun_out/summ16.log; exit 1; }
tail -3 gpurun_out/summ16.log
