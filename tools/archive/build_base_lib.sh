#!/bin/bash
# Build libfac_cvit.so of a git ref (default HEAD) into fac_fake_amd/libfac_cvit_base.so
# for same-box A/B runs: FAC_CVIT_LIB=$PWD/fac_fake_amd/libfac_cvit_base.so python bench.py ...
set -e
REF=${1:-HEAD}
R=$(git rev-parse --show-toplevel)
WT=/tmp/fac_base_wt
rm -rf $WT && git -C $R worktree prune && git -C $R worktree add -f --detach $WT $REF > /dev/null
(cd $WT && python -c "from fac_fake_amd import build; build.build()" > /dev/null)
cp $WT/fac_fake_amd/libfac_cvit.so $R/fac_fake_amd/libfac_cvit_base.so
git -C $R worktree remove --force $WT
echo "built $REF -> fac_fake_amd/libfac_cvit_base.so"
