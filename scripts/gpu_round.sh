#!/bin/bash
# One GPU call: smoke + GPU tests + default bench, then rocprofv3 evidence for the
# default 1 GiB workload (trace + FETCH/WRITE passes) under tag $1.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r02}
bash scripts/gpu_check.sh || exit 1
bash scripts/profile.sh "$TAG" || exit 1
python3 scripts/summarize_profile.py "$TAG" > gpurun_out/summ.log 2>&1 || { tail -5 gpurun_out/summ.log; exit 1; }
tail -3 gpurun_out/summ.log
