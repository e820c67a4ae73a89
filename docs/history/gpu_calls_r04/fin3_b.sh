# Round 4 closing measurement, part B: PMC records and bench lines of the other BASELINE configs,
# scaling probe, Table 1
bash tools/pmc_configs.sh r4fin3 && bash tools/round_measure.sh r4fin3 B
