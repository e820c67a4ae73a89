#!/bin/bash
# PMC counter passes over a short bench run (run on the GPU box).  One rocprofv3 invocation per
# counter group (no tracing domains mixed in).  Stops at the first crash/timeout exit status.
# usage: tools/pmc.sh TAG GROUPFILE [extra bench args]      (GROUPFILE: one counter group per line)
TAG=$1; GROUPS_FILE=$2; shift 2
export TMPDIR=/tmp
mkdir -p gpurun_out
# exactly one rendered pass: --no-extras skips the event, counter, full-frame and parity legs
BENCH="python3 bench.py --steps 1 --warmup 0 --no-extras $*"
i=0
while read -r GROUP; do
  [ -z "$GROUP" ] && continue
  case $GROUP in \#*) continue;; esac
  i=$((i+1))
  timeout -k 10 150 rocprofv3 --pmc $GROUP -d gpurun_out/pmc_${TAG}_$i -o run --output-format csv -- $BENCH > gpurun_out/pmc_${TAG}_$i.log 2>&1
  rc=$?
  echo "group $i rc=$rc: $GROUP"
  case $rc in 0) ;; *) echo "stopping after rc=$rc"; tail -5 gpurun_out/pmc_${TAG}_$i.log; exit $rc;; esac
done < "$GROUPS_FILE"
