#!/bin/bash
# Build an experiment variant of libgradtts.so with extra -D flags on every source.
# usage: tools/build_variant.sh <name> [-DFLAG ...]   -> ab/<name>/libgradtts.so
set -e
NAME=$1; shift
R=$(cd $(dirname $0)/.. && pwd)
D=$R/ab/$NAME; mkdir -p $D
# PK="" builds with the compiler's packed-fp32 instructions (the product build disables them, build.py)
PK=${PK--Xclang -target-feature -Xclang -packed-fp32-ops}
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I $R/include -I $R/grad-tts_amd/csrc -Wno-unused-result $PK"
SRCS=$(cd $R/grad-tts_amd/csrc && ls *.hip *.cpp | grep -v torch_ops)   # (every library source, as build.py)
for s in $SRCS; do
  L=""; case $s in *.cpp) L="-x hip";; conv64.hip) L="-mllvm -pragma-unroll-threshold=1000000";; esac   # (build.py SRC_FLAGS)
  /opt/rocm/bin/hipcc $F "$@" $L -c $R/grad-tts_amd/csrc/$s -o $D/$s.o 2>&1 | grep -v "packed-fp32-ops" || true &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/libgradtts.so $(for s in $SRCS; do echo $D/$s.o; done)
rm -f $D/*.o
echo built $D/libgradtts.so
