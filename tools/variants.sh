#!/bin/bash
# Build A/B variants of librtamd.so under build_var/<name> (here, on the CPU container).
# usage: tools/variants.sh "name:-DX=1 -DY=2" ...
cd "$(dirname "$0")/.."
for spec in "$@"; do
  name=${spec%%:*}; defs=${spec#*:}
  make -s -C cuda-raytracer_amd OUT=$(pwd)/cuda-raytracer_amd/build_var/$name EXTRA_DEFS="$defs" $(pwd)/cuda-raytracer_amd/build_var/$name/librtamd.so || exit 1
  echo "built $name ($defs)"
done
