# Round 4 second closing measurement (after the kids mask, shade round trips, PCG and nontemporal radiance
# stores), part A (HEAD in .rev): GPU suite, smoke, PMC passes of one teapot pass, bench lines, kernel trace
bash tools/round_measure.sh r4fin2 A
