#!/bin/bash
# Round 6: status strides, longer A/B. RL encode runs32 at 1 GiB / 4 GiB / 256 MiB
# (strides 16 / 4 / 2), FL encode u8 and lo4 at 1 GiB and u8 16 GiB (16 / 4 / 2),
# and FETCH_SIZE of the FL encode per launch.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06_stride2
mkdir -p $O
A=scripts/ab_libs
for nb in 1073741824 4294967296 268435456; do
  timeout -k 10 200 python -u scripts/ab_libs.py --op rl_encode --libs $A/libflrl_cur.so,$A/libflrl_st4.so,$A/libflrl_st2.so --kind runs32 --bytes $nb --reps 60 > $O/rl_$nb.log 2>&1 || { echo "fail rl $nb"; tail -5 $O/rl_$nb.log; exit 1; }
  tail -4 $O/rl_$nb.log
done
for k in u8 lo4; do
  timeout -k 10 200 python -u scripts/ab_libs.py --op fl_encode --libs $A/libflrl_cur.so,$A/libflrl_fst4.so,$A/libflrl_fst2.so --kind $k --reps 40 > $O/fl_$k.log 2>&1 || { echo "fail fl $k"; tail -5 $O/fl_$k.log; exit 1; }
  tail -4 $O/fl_$k.log
done
timeout -k 10 300 python -u scripts/ab_libs.py --op fl_encode --libs $A/libflrl_cur.so,$A/libflrl_fst4.so,$A/libflrl_fst2.so --kind u8 --bytes 17179869184 --reps 10 > $O/fl_16g.log 2>&1 || { echo "fail fl 16g"; tail -5 $O/fl_16g.log; exit 1; }
tail -4 $O/fl_16g.log
for b in cur fst4 fst2; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f_$b -o run -- python3 scripts/ab_libs.py --op fl_encode --libs $A/libflrl_$b.so --kind u8 --reps 4 > $O/f_$b.log 2>&1 || { echo "pmc $b failed"; exit 1; }
  python3 - "$O/f_$b" "$b" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True)[0]
v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if "fl_encode" in r["Kernel_Name"] and r["Counter_Name"] == "FETCH_SIZE"]
print(sys.argv[2], "FL encode FETCH_SIZE KiB per launch (raw):", [round(x) for x in v[-3:]])
PY
done
