#!/bin/bash
# Experiment variant of libgradtts.so that recompiles ONE source with extra -D flags and links it with the tree's
# other objects (grad-tts_amd/csrc/_obj, from build.py).   usage: tools/build_variant1.sh <src.hip> <name> [-DFLAG ...]
# (SRCFILE=path: compile that file in place of csrc/<src.hip>, e.g. an older revision)
set -e
SRC=$1; NAME=$2; shift 2
R=$(cd $(dirname $0)/.. && pwd)
D=$R/ab/$NAME; mkdir -p $D
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I $R/include -I $R/grad-tts_amd/csrc -Wno-unused-result -Xclang -target-feature -Xclang -packed-fp32-ops"
[ "$SRC" = conv64.hip ] && F="$F -mllvm -pragma-unroll-threshold=1000000"   # as build.py SRC_FLAGS
/opt/rocm/bin/hipcc $F "$@" -c ${SRCFILE:-$R/grad-tts_amd/csrc/$SRC} -o $D/$SRC.o 2>&1 | grep -v "packed-fp32-ops" || true
OBJS=$(ls $R/grad-tts_amd/csrc/_obj/*.o | grep -v "/$SRC.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/libgradtts.so $OBJS $D/$SRC.o
rm -f $D/$SRC.o
echo built $D/libgradtts.so
