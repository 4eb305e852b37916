#!/bin/bash
# Build an A/B variant of libbote_hip.so with extra compiler flags:
#   scripts/build_variant.sh NAME "-DFOO=1"   ->  fantoch_amd/lib_NAME/libbote_hip.so
# Use it with BOTE_LIB_PATH=fantoch_amd/lib_NAME/libbote_hip.so (timing experiments only).
set -e
NAME=$1; FLAGS=$2
D=fantoch_amd/lib_$NAME
mkdir -p $D/obj
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wno-unused-result $FLAGS"
# GROUP_SRC: an alternative bote_group.hip (e.g. `git show HEAD:...` for an A/B of the committed kernel)
for f in bote_kernels bote_sweep bote_group bote_quorums bote_chain bote_capi; do
  src=fantoch_amd/csrc/$f.hip
  if [ "$f" = bote_group ] && [ -n "${GROUP_SRC:-}" ]; then src=$GROUP_SRC; fi
  # rebuild when the object is missing or older than its source or any shared
  # header (a stale object with an old FastArgs layout faults on the device)
  stale=0
  [ "$f" = bote_group ] && stale=1
  [ -f $D/obj/$f.o ] || stale=1
  for dep in $src fantoch_amd/csrc/*.hpp include/bote_hip.h; do
    [ -f $D/obj/$f.o ] && [ "$dep" -nt $D/obj/$f.o ] && stale=1
  done
  if [ $stale = 1 ]; then $H -I fantoch_amd/csrc -c $src -o $D/obj/$f.o & fi
done
# host-only code (plain C++)
if [ ! -f $D/obj/bote_host.o ] || [ fantoch_amd/csrc/bote_host.cpp -nt $D/obj/bote_host.o ] || [ fantoch_amd/csrc/bote_host.hpp -nt $D/obj/bote_host.o ]; then
  g++ -O2 -std=c++17 -fPIC $FLAGS -c fantoch_amd/csrc/bote_host.cpp -o $D/obj/bote_host.o &
fi
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -Wl,--no-undefined -o $D/libbote_hip.so $D/obj/*.o
echo built $D/libbote_hip.so
# Device-assert variant (soft asserts):  scripts/build_variant.sh debug -DBOTE_DEBUG
