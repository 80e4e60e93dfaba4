#!/bin/bash
# Build the library of another git revision for same-box A/B runs (tools/lib_ab.sh):
#   bash tools/build_rev_lib.sh REV NAME   ->  tools/variants/libspecenh_NAME.so
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
REV=$1; NAME=$2
WT=/tmp/specenh_wt_$NAME
rm -rf $WT; git -C $R worktree prune
git -C $R worktree add --detach $WT $REV > /dev/null
(cd $WT && python3 -c "import sys; sys.path.insert(0, 'spectrogram-enhancement_amd'); import build; build.build(force=True, jobs=8)" > /dev/null)
mkdir -p $R/tools/variants
cp $WT/spectrogram-enhancement_amd/specenh/libspecenh.so $R/tools/variants/libspecenh_$NAME.so
git -C $R worktree remove --force $WT
echo $R/tools/variants/libspecenh_$NAME.so
