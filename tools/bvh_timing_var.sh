#!/bin/bash
# GPU BVH build times of librtamd.so variants (tools/variants.sh): usage tools/bvh_timing_var.sh NAME...
for v in "$@"; do
  echo "== $v"
  RTAMD_LIB=$PWD/cuda-raytracer_amd/build_var/$v/librtamd.so timeout -k 10 200 python tools/bvh_timing.py 2>&1 | grep gpu || exit 1
done
