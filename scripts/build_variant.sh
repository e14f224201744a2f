#!/bin/bash
# Build a variant of libflrl.so with extra compile flags for A/B timing
# (scripts/ab_libs.py), e.g.: bash scripts/build_variant.sh stage10k -DFLRL_RL_STAGE=10240
# (FLRL_TUNING_BUILD is defined here: csrc/flrl_tuning.hpp lists the overrides)
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=$ROOT/scripts/ab_libs/$NAME
mkdir -p "$OUT"
for f in flrl_common flrl_fl flrl_rl flrl_shard flrl_stream; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I"$ROOT/include" \
      -I"$ROOT/fl-rl-compression-mpi_amd/csrc" -DFLRL_TUNING_BUILD "$@" -c "$ROOT/fl-rl-compression-mpi_amd/csrc/$f.hip" -o "$OUT/$f.o" &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$ROOT/scripts/ab_libs/libflrl_$NAME.so" "$OUT"/*.o \
    -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -rf "$OUT"
echo "scripts/ab_libs/libflrl_$NAME.so"
