#!/bin/bash
# Kernel experiments: build ggrs_amd/var/lib_<name>.so = the product library with
# ops_exgame_p2.hip (ALLP=1: every ops_exgame_p<P>.hip) recompiled under extra -D
# flags; tools/varrun.sh benches them via GGRS_AMD_LIB.
# usage: tools/mkvar.sh <name> [-DFOO=1 ...]   (after a normal make)
set -e
cd "$(dirname "$0")/../ggrs_amd/csrc"
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -DRB_EXPERIMENTS=0 -mllvm -amdgpu-sched-strategy=max-ilp"
name=$1; shift
mkdir -p build/var ../var
TUS=${TUS:-ops_exgame_p2}; [ -n "$ALLP" ] && TUS="ops_exgame_p1 ops_exgame_p2 ops_exgame_p3 ops_exgame_p4"
VOBJS=""
for tu in $TUS; do
  /opt/rocm/bin/hipcc $F "$@" -c -o build/var/${tu}_$name.o $tu.hip &
  VOBJS="$VOBJS build/var/${tu}_$name.o"
done
wait
OBJS=$(ls build/*.o | grep -v -E "$(echo $TUS | tr ' ' '|')")
/opt/rocm/bin/hipcc $F -shared -o ../var/lib_$name.so $OBJS $VOBJS -ldl
