#!/bin/bash
# Build the library of a git revision (default HEAD) into ab/<name>/ for same-box A/B timing.
# usage: tools/build_ref.sh <name> [rev]
set -e
NAME=$1; REV=${2:-HEAD}
R=$(cd $(dirname $0)/.. && pwd)
W=$(mktemp -d /tmp/gt_ref.XXXX)
git -C $R worktree add -f $W $REV >/dev/null 2>&1
(cd $W && python grad-tts_amd/build.py >/dev/null)
mkdir -p $R/ab/$NAME && cp $W/grad-tts_amd/gradtts_amd/libgradtts.so $R/ab/$NAME/
git -C $R worktree remove --force $W
echo built $R/ab/$NAME/libgradtts.so from $REV
