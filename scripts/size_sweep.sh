#!/bin/bash
# rocprofv3 kernel trace of rl_decode on random bytes at several sizes: per-kernel
# means per size (does the decode's re-read of the counts hit the MALL when the
# counts fit in it?). GPU box.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for b in ${SIZES:-134217728 268435456 1073741824}; do
  rm -rf gpurun_out/sweep_$b
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sweep_$b/trace -o run -- \
      python3 scripts/ab_libs.py --op ${OP:-rl_decode} --libs fl-rl-compression-mpi_amd/lib/libflrl.so \
      --kind ${KIND:-u8} --bytes $b --reps 10 > gpurun_out/sweep_$b.log 2>&1 || { tail -5 gpurun_out/sweep_$b.log; exit 1; }
  echo "== $b"; grep "ms " gpurun_out/sweep_$b.log
  python3 scripts/pmc_summary.py gpurun_out/sweep_$b rl_
done
