#!/bin/bash
# Kernel experiments: build ggrs_amd/var/lib_<name>.so = the product library with
# ops_exgame.hip recompiled under extra -D flags (bench configuration only,
# RB_EXGAME_P2_ONLY); tools/varrun.sh benches them via GGRS_AMD_LIB.
# usage: tools/mkvar.sh <name> [-DFOO=1 ...]   (after a normal make)
# build variant libs: name + defines (ALLP=1: every ex_game player count, not only P = 2)
set -e
cd "$(dirname "$0")/../ggrs_amd/csrc"
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -DRB_EXPERIMENTS=0"
name=$1; shift
mkdir -p build/var ../var
P2ONLY="-DRB_EXGAME_P2_ONLY=1"; [ -n "$ALLP" ] && P2ONLY=""
/opt/rocm/bin/hipcc $F "$@" $P2ONLY -c -o build/var/ex_$name.o ops_exgame.hip
OBJS=$(ls build/*.o | grep -v ops_exgame.o)
/opt/rocm/bin/hipcc $F -shared -o ../var/lib_$name.so $OBJS build/var/ex_$name.o
