#!/bin/bash
# Round 6: RL encode status stride (FLRL_RL_STATUS_STRIDE granules per tile: 16 =
# one 128-B line, 8 = 64 B, 4 = 32 B) -- encode call time and FETCH_SIZE per launch.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06_stride
mkdir -p $O
L=${LIBS:-scripts/ab_libs/libflrl_cur.so,scripts/ab_libs/libflrl_st8.so,scripts/ab_libs/libflrl_st4.so}
for k in runs32 longruns zero upto12; do
  timeout -k 10 200 python -u scripts/ab_libs.py --op rl_encode --libs $L --kind $k --reps 30 > $O/$k.log 2>&1 || { echo "fail $k"; tail -5 $O/$k.log; exit 1; }
  tail -4 $O/$k.log
done
for b in ${PMCB:-cur st8 st4}; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f_$b -o run -- python3 scripts/ab_libs.py --op rl_encode --libs scripts/ab_libs/libflrl_$b.so --kind runs32 --reps 4 > $O/f_$b.log 2>&1 || { echo "pmc $b failed"; exit 1; }
  python3 - "$O/f_$b" "$b" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True)[0]
v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if "rl_encode_wave" in r["Kernel_Name"] and r["Counter_Name"] == "FETCH_SIZE"]
print(sys.argv[2], "FETCH_SIZE KiB per launch (raw, x2 for bytes read):", [round(x) for x in v[-3:]])
PY
done
