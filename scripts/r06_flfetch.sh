#!/bin/bash
# Round 6: new GPU tests (failed rank call between good calls without sync,
# bounded staging pool), then where the FL encode's extra fetch comes from:
# the shipped kernel against a PMC/timing build with static tile offsets
# (FLRL_FL_STATIC_W: no look-back status traffic), 1 GiB u8 and lo4.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06b
mkdir -p $O
timeout -k 10 60 rocprofv3 --list-avail > $O/avail.txt 2>&1 || echo "list-avail rc=$?"
timeout -k 10 400 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread \
    -k "without_sync or large_file or alternating or release_staging or runtime_failure" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
B=scripts/ab_libs/libflrl_base.so
timeout -k 10 200 python -u scripts/ab_libs.py --op fl_encode --libs $B,scripts/ab_libs/libflrl_static8.so --kind u8 --reps 20 > $O/ab_u8.log 2>&1 || { echo "ab u8 failed"; tail -5 $O/ab_u8.log; exit 1; }
tail -3 $O/ab_u8.log
timeout -k 10 200 python -u scripts/ab_libs.py --op fl_encode --libs $B,scripts/ab_libs/libflrl_static4.so --kind lo4 --reps 20 > $O/ab_lo4.log 2>&1 || { echo "ab lo4 failed"; tail -5 $O/ab_lo4.log; exit 1; }
tail -3 $O/ab_lo4.log
for v in "u8 base $B" "u8 static8 scripts/ab_libs/libflrl_static8.so" "lo4 base $B" "lo4 static4 scripts/ab_libs/libflrl_static4.so"; do
  set -- $v
  NOPMC= PMC_GROUPS="FETCH_SIZE;WRITE_SIZE" bash scripts/pmc_ab.sh fl_encode $1 $3 fl_$1_$2 > $O/pmc_$1_$2.log 2>&1 || { echo "pmc $1 $2 failed"; tail -5 $O/pmc_$1_$2.log; exit 1; }
  echo "== $1 $2"; grep -A3 fl_encode $O/pmc_$1_$2.log
done
