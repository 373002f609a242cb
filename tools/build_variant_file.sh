#!/bin/bash
# Experiment variant of libgradtts.so from an alternative copy of ONE source (e.g. the last commit's version, for a same-box
# A/B), linked with the tree's other objects.   usage: tools/build_variant_file.sh <file.hip> <tree-src-name> <name> [-D...]
set -e
FILE=$1; SRC=$2; NAME=$3; shift 3
R=$(cd $(dirname $0)/.. && pwd)
D=$R/ab/$NAME; mkdir -p $D
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I $R/include -I $R/grad-tts_amd/csrc -Wno-unused-result -Xclang -target-feature -Xclang -packed-fp32-ops"
/opt/rocm/bin/hipcc $F "$@" -x hip -c $FILE -o $D/$SRC.o 2>&1 | grep -v "packed-fp32-ops" || true
OBJS=$(ls $R/grad-tts_amd/csrc/_obj/*.o | grep -v "/$SRC.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/libgradtts.so $OBJS $D/$SRC.o
rm -f $D/$SRC.o
echo built $D/libgradtts.so
