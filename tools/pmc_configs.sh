#!/bin/bash
# PMC traffic and instruction counts of one rendered pass for the other BASELINE configs (run on the
# GPU box), recorded under each config's workload name in profiles/pmc_traffic.json and
# profiles/pmc_issue.json, which bench.py reads for roofline.traffic / .frame / .valu.
# usage: tools/pmc_configs.sh TAG            (each GPU step under its own limit inside tools/pmc.sh)
TAG=$1
export TMPDIR=/tmp
REV=$(cat .rev 2>/dev/null || echo unknown)
mkdir -p gpurun_out/$TAG
for cfg in cornell_plus lamp teapot:--no-sort lamp:--no-sort; do
  args="--scene $(echo $cfg | tr ':' ' ')"; name=$(echo $cfg | tr -d ':-')
  # the workload key exactly as bench.py names it
  wl=$(python3 - $args <<'EOF'
import sys
sys.argv = ["bench.py"] + sys.argv[1:]
import argparse
scene = sys.argv[sys.argv.index("--scene") + 1]
CONFIGS = {
    "teapot": ("teapot.scene", 1920, 1080, 2048, 16, True),
    "cornell_plus": ("cornell_plus.scene", 512, 512, 256, 8, True),
    "spheres": ("spheres.scene", 1024, 1024, 1024, 8, True),
    "lamp": ("lamp_available.scene", 1920, 1080, 4096, 32, True),
    "cornell": ("cornell.scene", 256, 256, 64, 4, True),
}
f, w, h, spp, b, sort = CONFIGS[scene]
if "--no-sort" in sys.argv:
    sort = False
print("%s %dx%d %dspp %d bounces sort=%s" % (f, w, h, spp, b, "on" if sort else "off"))
EOF
)
  echo "== $cfg: $wl $(date +%T)"
  bash tools/pmc.sh ${TAG}_${name}_tf tools/pmc_groups/traffic.txt $args > gpurun_out/$TAG/pmc_tf_$name.log 2>&1 || { cat gpurun_out/$TAG/pmc_tf_$name.log; exit 1; }
  python3 tools/pmc_summary.py ${TAG}_${name}_tf --json profiles/pmc_traffic.json --workload "$wl" \
      --run "rev $REV: python3 bench.py --steps 1 --warmup 0 --no-extras $args (tools/pmc.sh ${TAG}_${name}_tf)" \
      > gpurun_out/$TAG/pmc_summary_$name.txt || exit 1
  bash tools/pmc.sh ${TAG}_${name}_st tools/pmc_groups/stall.txt $args > gpurun_out/$TAG/pmc_st_$name.log 2>&1 || { cat gpurun_out/$TAG/pmc_st_$name.log; exit 1; }
  python3 tools/stall_summary.py ${TAG}_${name}_st --json profiles/pmc_issue.json --workload "$wl" \
      --run "rev $REV: python3 bench.py --steps 1 --warmup 0 --no-extras $args (tools/pmc.sh ${TAG}_${name}_st)" \
      > gpurun_out/$TAG/pmc_stall_$name.txt || exit 1
done
cp profiles/pmc_traffic.json profiles/pmc_issue.json gpurun_out/$TAG/
echo done
