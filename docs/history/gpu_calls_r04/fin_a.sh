# Round 4 closing measurement, part A (HEAD in .rev): GPU suite, smoke, PMC passes of one teapot pass, bench lines, kernel trace
bash tools/round_measure.sh r4fin A
