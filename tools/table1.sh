#!/bin/bash
# REPORT.pdf Table 1 setup (1000x1000, 10 bounces, 1/10/100 spp, sort and no_sort) through the
# drop-in CLI on one MI355X: the CLI's own "GPU Took" line (the reference's timed span,
# raytracing.cu:172-281), next to the published GTX 1080 numbers.
# lamp uses lamp_available.scene (two meshes are missing upstream); teapot/lamp use the
# procedural stand-in env map.  Run on the GPU box: tools/table1.sh OUTFILE
OUT=${1:-gpurun_out/table1.txt}
BIN=$(pwd)/cuda-raytracer_amd/build/raytracing
cd assets || exit 1
echo "scene spp mode gpu_took_s" > ../$OUT
for scene in spheres cornell cornell_plus teapot glass_teapot lamp_available; do
  for spp in 1 10 100; do
    for mode in sort no_sort; do
      extra=""; [ $mode = no_sort ] && extra=no_sort
      line=$(timeout -k 10 120 $BIN $scene.scene $extra --image 1000 1000 $spp 10 1 --out /tmp/t1.png 2>>../$OUT.timing | grep "GPU Took") || { echo "failed: $scene $spp $mode"; exit 1; }
      echo "$scene $spp $mode $(echo $line | awk '{print $3}' | tr -d s)" >> ../$OUT
    done
  done
done
cat ../$OUT
