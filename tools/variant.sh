#!/bin/bash
# Builds an experimental variant of the package into variants/NAME/diff_gaussian_sampling
# (git-ignored; travels to the GPU box with gpurun) with extra hipcc flags, for A/B timing with
# tools/ab.py.   usage: tools/variant.sh NAME "-DFOO=1 ..."
set -eu
REPO=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; FLAGS=${2:-}
OUT=$REPO/variants/$NAME
mkdir -p "$OUT/diff_gaussian_sampling" "$OUT/build"
cp "$REPO"/diff-gaussian-sampling_amd/diff_gaussian_sampling/*.py "$OUT/diff_gaussian_sampling/"
DGS_PKG_OUT=$OUT/diff_gaussian_sampling DGS_OBJ_OUT=$OUT/build DGS_EXTRA_CFLAGS="$FLAGS" \
    python "$REPO/diff-gaussian-sampling_amd/build.py"
rm -rf "$OUT/build"
