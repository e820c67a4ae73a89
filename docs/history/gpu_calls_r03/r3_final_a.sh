# Round 3 closing measurement, part A (tests, smoke, PMC records, teapot lines, kernel trace)
export TMPDIR=/tmp
bash tools/round_measure.sh r3fin A
