#!/bin/bash
# A/B helper: build librspl.so from a git revision (default HEAD) in a scratch worktree and copy it
# in-tree as rspl-slam_amd/librspl_base.so (RSPL_LIB=librspl_base.so selects it).
set -e
REV=${1:-HEAD}
R=$(cd "$(dirname "$0")/.." && pwd)
W=/tmp/rspl_base_wt
rm -rf $W
git -C $R worktree prune
git -C $R worktree add -f --detach $W $REV > /dev/null
make -s -j8 -C $W/rspl-slam_amd/csrc > /dev/null
cp $W/rspl-slam_amd/librspl.so $R/rspl-slam_amd/librspl_base.so
git -C $R worktree remove --force $W
echo "librspl_base.so <- $(git -C $R rev-parse --short $REV)"
