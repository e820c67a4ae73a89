#!/bin/bash
# Build librtamd.so of a git revision into cuda-raytracer_amd/build_var/<name> (for tools/ab.py).
# usage: tools/build_rev.sh NAME REV ["-DX=1 ..."]
cd "$(dirname "$0")/.."
NAME=$1; REV=$2; DEFS=$3
SRC=cuda-raytracer_amd/build_var/_src_$NAME
rm -rf "$SRC"; mkdir -p "$SRC"
git archive "$REV" cuda-raytracer_amd include | tar -x -C "$SRC" || exit 1
make -s -C "$SRC/cuda-raytracer_amd" OUT=$(pwd)/cuda-raytracer_amd/build_var/$NAME EXTRA_DEFS="$DEFS" \
  $(pwd)/cuda-raytracer_amd/build_var/$NAME/librtamd.so || exit 1
rm -rf "$SRC"
echo "built $NAME from $(git rev-parse --short $REV)"
