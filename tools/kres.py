"""Per-kernel resource usage (VGPRs, SGPRs, LDS, scratch, occupancy bound) from a gfx950 .s file.
usage: python tools/kres.py file.s"""
import re
import sys

txt = open(sys.argv[1]).read()
for m in re.finditer(r"\.amdhsa_kernel (\S+)(.*?)\.end_amdhsa_kernel", txt, re.S):
    name, body = m.group(1), m.group(2)
    g = lambda k: int(re.search(r"\.%s (\d+)" % k, body).group(1))
    v, s, lds, scr = g("amdhsa_next_free_vgpr"), g("amdhsa_next_free_sgpr"), \
        g("amdhsa_group_segment_fixed_size"), g("amdhsa_private_segment_fixed_size")
    short = re.sub(r"_ZN12_GLOBAL__N_1\d+", "", name)
    short = re.sub(r"EEEv.*|Ev.*|E[PN].*", "", short)
    waves = min(8, 512 // max(8, (v + 7) // 8 * 8))
    print("%-40s vgpr %3d sgpr %3d lds %6d scratch %4d  waves/SIMD(vgpr) %d" % (short, v, s, lds, scr, waves))
