# Round 4 closing measurement at the session's final kernel (rt_render.hip as at 1645831; HEAD in .rev),
# part A: GPU suite, smoke, PMC passes of one teapot pass, bench lines, kernel trace
bash tools/round_measure.sh r4fin3 A
