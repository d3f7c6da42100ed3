#!/bin/bash
# build librlamd with one env's TU (TU=frozen_lake | cliff_walking | taxi | blackjack |
# frozen_lake_edited; default frozen_lake) compiled under -DRLAMD_EXP=<mask> (or
# $VARIANT_FLAG=<v>) into rl-rust_amd/exp/librlamd_<mask>.so, the other TUs from
# build/.  Timing experiments only: masked variants may compute WRONG results.
set -e
cd "$(dirname "$0")/../rl-rust_amd"
mkdir -p exp
TU=${TU:-frozen_lake}
ALL="frozen_lake cliff_walking taxi blackjack frozen_lake_edited"
for m in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../include -fPIC -ffp-contract=off -fno-fast-math -Wall \
     -Wno-unused-result -mllvm -amdgpu-atomic-optimizer-strategy=None ${VARIANT_FLAG:--DRLAMD_EXP}=$m \
     -c csrc/rl_train_$TU.hip -o exp/tu_$m.o &
done
wait
for m in "$@"; do
  objs="exp/tu_$m.o"
  for t in $ALL; do [ "$t" = "$TU" ] || objs="$objs build/rl_train_$t.hip.o"; done
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o exp/librlamd_$m.so $objs \
     build/rl_misc.hip.o build/rl_host.cpp.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
done
rm -f exp/*.o
ls -la exp
