#!/bin/bash
# r05 closing measurement, part B: PMC records of the other configs, then their bench lines, the strong-scaling
# probes (torch.distributed path and the in-library path) and REPORT.pdf Table 1.
export TMPDIR=/tmp
bash tools/pmc_configs.sh r5fin > gpurun_out/r5fin_pmc_configs.log 2>&1 || { tail -20 gpurun_out/r5fin_pmc_configs.log; exit 1; }
tail -2 gpurun_out/r5fin_pmc_configs.log
bash tools/round_measure.sh r5fin B || exit 1
timeout -k 10 600 python tools/share_probe.py 13 26 > gpurun_out/r5fin/share_probe.txt 2>&1 || { tail gpurun_out/r5fin/share_probe.txt; exit 1; }
cat gpurun_out/r5fin/share_probe.txt
