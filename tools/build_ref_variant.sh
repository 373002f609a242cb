#!/bin/bash
# Build libgradtts.so from a git revision's sources into ab/<name> (same-box A/B against an earlier commit).
# usage: tools/build_ref_variant.sh <name> <rev> [-DFLAG ...]
set -e
NAME=$1; REV=$2; shift 2
R=$(cd $(dirname $0)/.. && pwd)
SRC=$(mktemp -d)
git -C $R archive $REV grad-tts_amd/csrc include | tar -x -C $SRC
D=$R/ab/$NAME; mkdir -p $D
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I $SRC/include -I $SRC/grad-tts_amd/csrc -Wno-unused-result -Xclang -target-feature -Xclang -packed-fp32-ops"
SRCS=$(cd $SRC/grad-tts_amd/csrc && ls *.hip *.cpp | grep -v torch_ops)
for s in $SRCS; do
  L=""; case $s in *.cpp) L="-x hip";; conv64.hip) L="-mllvm -pragma-unroll-threshold=1000000";; esac   # (build.py SRC_FLAGS)
  /opt/rocm/bin/hipcc $F "$@" $L -c $SRC/grad-tts_amd/csrc/$s -o $D/$s.o 2>&1 | grep -v "packed-fp32-ops\|warning" || true &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $D/libgradtts.so $(for s in $SRCS; do echo $D/$s.o; done)
rm -f $D/*.o; rm -rf $SRC
echo built $D/libgradtts.so from $REV
