#!/bin/bash
# Experiment build: rl-rust_amd/exp/librlamd_<name>.so with ONE env TU compiled for
# ONE kernel instantiation (-DRLAMD_ONLY=ag,po,se,al,pr) from the current sources,
# plus rl_misc / rl_host from the current sources (the LDS carve and the host agree);
# the other env TUs are compiled empty (no kernels: a small .so to ship).  Timing and
# targeted parity only.
#   NAME=rowmax TU=frozen_lake ONLY=0,0,0,1,0 EXTRA="-DRLAMD_ROWMAX=0" scripts/build_fast.sh
set -e
cd "$(dirname "$0")/../rl-rust_amd"
mkdir -p exp
TU=${TU:-frozen_lake}
NAME=${NAME:-fast}
ONLY=${ONLY:-0,0,0,1,0}
ALL="frozen_lake cliff_walking taxi blackjack frozen_lake_edited"
SRC=${SRCDIR:-csrc}       # SRCDIR / INCDIR: a patched copy of the sources (diagnostic builds)
INC=${INCDIR:-../include}
F="--offload-arch=gfx950 -O3 -std=c++17 -I$INC -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-result -mllvm -amdgpu-atomic-optimizer-strategy=None"
/opt/rocm/bin/hipcc $F -DRLAMD_ONLY=$ONLY $EXTRA -c $SRC/rl_train_$TU.hip -o exp/tu_$NAME.o &
/opt/rocm/bin/hipcc $F $EXTRA -c $SRC/rl_misc.hip -o exp/misc_$NAME.o &
/opt/rocm/bin/hipcc $F $EXTRA -DRLAMD_BUILD_FLAGS='"exp '"$NAME $EXTRA"'"' -c $SRC/rl_host.cpp -o exp/host_$NAME.o &
printf 'const char *rl_build_id(void) { return "exp:%s"; }\n' "$NAME" > exp/id_$NAME.c
gcc -O2 -fPIC -c exp/id_$NAME.c -o exp/id_$NAME.o
objs="exp/tu_$NAME.o exp/misc_$NAME.o exp/host_$NAME.o exp/id_$NAME.o"
for t in $ALL; do
  [ "$t" = "$TU" ] && continue
  /opt/rocm/bin/hipcc $F -DRLAMD_ONLY=9,9,9,9,9 -c $SRC/rl_train_$t.hip -o exp/empty_${NAME}_$t.o &
  objs="$objs exp/empty_${NAME}_$t.o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o exp/librlamd_$NAME.so $objs -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -f exp/tu_$NAME.o exp/misc_$NAME.o exp/host_$NAME.o exp/empty_${NAME}_*.o exp/id_$NAME.[co]
ls -la exp/librlamd_$NAME.so
