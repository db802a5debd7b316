#!/bin/bash
# Build a variant of libsbeacon_hip.so for A/B runs (tools/req_tune.py with
# SBEACON_LIB=...): tools/build_variant.sh NAME [git-rev] [extra hipcc flags...]
# -- the csrc of git-rev (default: the working tree), compiled with the
# product flags plus the extras, into tools/variants/NAME/libsbeacon_hip.so.
set -e
NAME=$1; REV=${2:-WORKTREE}; shift 2 || shift $#
R=$(cd "$(dirname "$0")/.." && pwd)
W=/tmp/sbeacon_variant_$NAME
rm -rf $W && mkdir -p $W/pkg/csrc $W/include
if [ "$REV" = WORKTREE ]; then
  cp $R/terraform-aws-serverless-beacon_amd/csrc/* $W/pkg/csrc/; cp $R/include/sbeacon.h $W/include/
else
  for f in $(git -C $R ls-tree --name-only $REV terraform-aws-serverless-beacon_amd/csrc/); do
    git -C $R show $REV:$f > $W/pkg/csrc/$(basename $f); done
  git -C $R show $REV:include/sbeacon.h > $W/include/sbeacon.h
fi
# SED: an optional sed script applied to the variant's query_kernels.hip
# (timing ablations: e.g. SED='s/^    if (nch) {$/    if (false) {/' skips
# request_eval_kernel's candidate loop -- wrong answers, counters only)
if [ -n "$SED" ]; then sed -i -e "$SED" $W/pkg/csrc/query_kernels.hip; fi
FL="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I$W/include $*"
objs=""
for s in $(ls $W/pkg/csrc | grep -E "\.(cpp|hip)$" | grep -v synth.cpp); do
  x=""; case $s in *.cpp) x="-x hip";; esac
  /opt/rocm/bin/hipcc $x $FL -c $W/pkg/csrc/$s -o $W/$s.o &
  objs="$objs $W/$s.o"
done
wait
mkdir -p $R/tools/variants/$NAME
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $R/tools/variants/$NAME/libsbeacon_hip.so $objs -lz -lpthread
echo $R/tools/variants/$NAME/libsbeacon_hip.so
