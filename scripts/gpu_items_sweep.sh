#!/bin/bash
# A/B of FL tile sizes (ITEMS = 16-byte chunks per lane) in one box session.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for e in 16 8 4; do for d in 16 8 4; do
  FLRL_FL_ENC_ITEMS=$e FLRL_FL_DEC_ITEMS=$d timeout -k 10 120 python bench.py --steps 20 --warmup 3 --cpu-sample 0 > gpurun_out/sweep_${e}_${d}.log 2>&1 || { echo "fail $e $d"; tail -5 gpurun_out/sweep_${e}_${d}.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('gpurun_out/sweep_${e}_${d}.log').read().strip().splitlines()[-1]);k=d['kernels'];print('enc',$e,'dec',$d,'step',d['ms_per_step'],'enc',k['fl_encode'],'dec',k['fl_decode'],'copy',k['device_copy_ceiling']['GBps'],'rt',d['parity']['roundtrip'])"
done; done
