#!/bin/bash
# build librlamd with the FrozenLake TU compiled under -DRLAMD_EXP=<mask> (or $VARIANT_FLAG=<v>; timing
# experiments only: the masked variants compute WRONG results) into rl-rust_amd/exp/
set -e
cd "$(dirname "$0")/../rl-rust_amd"
mkdir -p exp
for m in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../include -fPIC -ffp-contract=off -fno-fast-math -Wall \
     -Wno-unused-result -mllvm -amdgpu-atomic-optimizer-strategy=None ${VARIANT_FLAG:--DRLAMD_EXP}=$m -c csrc/rl_train_frozen_lake.hip -o exp/fl_$m.o &
done
wait
for m in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o exp/librlamd_$m.so exp/fl_$m.o \
     build/rl_train_cliff_walking.hip.o build/rl_train_taxi.hip.o build/rl_train_blackjack.hip.o \
     build/rl_train_frozen_lake_edited.hip.o build/rl_misc.hip.o build/rl_host.cpp.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
done
rm -f exp/*.o
ls -la exp
