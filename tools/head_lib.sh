#!/bin/bash
# Build libldpc_nms.so of a git revision (default HEAD) in a scratch worktree, for A/B runs of
# the working tree against it:  bash tools/head_lib.sh ab_libs/head.so [REV]
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=$(realpath -m "$1"); REV=$(git rev-parse "${2:-HEAD}")
W=/tmp/ldpc_headtree
if [ -d $W ]; then git -C $W checkout -q --detach "$REV"; else git worktree add -q --detach $W "$REV"; fi
(cd $W && python -m ldpc_error_floor_amd.build --jobs 8 > /tmp/ldpc_headtree_build.log 2>&1)
mkdir -p "$(dirname "$OUT")"
cp $W/ldpc_error_floor_amd/libldpc_nms.so "$OUT"
echo "$OUT ($(git -C $W rev-parse --short HEAD))"
