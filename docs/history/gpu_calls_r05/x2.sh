#!/bin/bash
# r05: XCD-affine trace order, per launch: exclusive launch A/B and bounce-1 fabric bytes (PMC).
export TMPDIR=/tmp
OUT=gpurun_out/r5_x2; mkdir -p $OUT
echo "== launch ab $(date +%T)"
timeout -k 10 600 python tools/launch_ab.py 3 noxc default default@RTAMD_XCDA=16 > $OUT/launch_ab.txt 2>&1 || { tail $OUT/launch_ab.txt; exit 1; }
tail -4 $OUT/launch_ab.txt
for v in noxc default; do
  lib=$PWD/cuda-raytracer_amd/build_var/$v/librtamd.so; [ $v = default ] && lib=$PWD/cuda-raytracer_amd/build/librtamd.so
  echo "== pmc $v $(date +%T)"
  RTAMD_LIB=$lib bash tools/pmc.sh r5x2_$v tools/pmc_groups/traffic.txt > $OUT/pmc_$v.log 2>&1 || { cat $OUT/pmc_$v.log; exit 1; }
  python3 tools/pmc_summary.py r5x2_$v --json $OUT/pmc_$v.json --workload teapot > $OUT/pmc_summary_$v.txt || exit 1
  python3 -c "import json;d=json.load(open('$OUT/pmc_$v.json'))['teapot'];print('$v bytes by launch (GB):',[round(x/1e9,3) for x in d['trace_bytes_by_launch'][:4]],'dur',d['trace_dur_ms_per_launch'][:4])"
done
