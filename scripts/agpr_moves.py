"""Per kernel: MFMAs and AGPR<->VGPR copies inside loops of a hipcc -S listing (blocks the
compiler annotates 'Loop Header' / 'in Loop').  Copies in a loop usually mean loop-carried
accumulators the allocator left in VGPRs (fix: fa::pin_agpr).
usage: python scripts/agpr_moves.py file.s [name-filter]"""
import re
import sys

s = open(sys.argv[1]).read()
flt = sys.argv[2] if len(sys.argv) > 2 else ""
for m in re.finditer(r"^(_Z\w+):", s, re.M):
    name = m.group(1)
    if flt not in name:
        continue
    body = s[m.end():s.index(".Lfunc_end", m.end())]
    inloop = False
    mf = mv = 0
    for line in body.split("\n"):
        if re.match(r"^\.LBB\w+:", line):
            inloop = "Loop" in line
            continue
        if inloop:
            if "v_mfma" in line:
                mf += 1
            elif "v_accvgpr_read" in line or "v_accvgpr_write" in line:
                mv += 1
    if mf:
        print(f"{name[:90]:90s} loop_mfma={mf:4d} loop_agpr_copies={mv:4d}")
