#!/bin/bash
# Host-buffer API probe (GPU box): parallel first-touch scaling of malloc'd
# memory, then flrl_fl_compress/decompress rates for the shipped library and
# variant builds (scripts/ab_libs/libflrl_<name>.so copied over the in-tree one
# in this disposable copy of the tree).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ "${TOUCH:-1}" = 1 ]; then ./scripts/touch_probe.bin 2048 16 1 && ./scripts/touch_probe.bin 2048 16 0 || exit 1; fi
cp fl-rl-compression-mpi_amd/lib/libflrl.so /tmp/libflrl_ship.so
for v in ship $VARIANTS; do
  if [ "$v" = ship ]; then cp /tmp/libflrl_ship.so fl-rl-compression-mpi_amd/lib/libflrl.so; else cp scripts/ab_libs/libflrl_$v.so fl-rl-compression-mpi_amd/lib/libflrl.so; fi
  echo "== $v"
  timeout -k 10 300 python3 scripts/bench_stream.py --mem-only --bytes 2147483648 --reps 3 > gpurun_out/host_$v.json 2> gpurun_out/host_$v.err || { tail -5 gpurun_out/host_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/host_$v.json')); print({k: v for k, v in d.items() if 'GBps' in k})"
  grep -h "host-prof" gpurun_out/host_$v.err | tail -4 || true
done
