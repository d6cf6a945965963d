"""Per-kernel register / spill / occupancy table from `hipcc -Rpass-analysis=kernel-resource-usage`.
usage: hipcc ... -Rpass-analysis=kernel-resource-usage 2>&1 | python scripts/kres.py [filter]"""
import re
import sys

flt = sys.argv[1] if len(sys.argv) > 1 else ""
cur = None
rows = []
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+([A-Za-z /\[\]]+): (\d+)", line)
    if m and cur is not None:
        cur[m.group(1).strip()] = int(m.group(2))
for r in rows:
    if flt in r["name"]:
        print(f"{r['name'][:90]:90s} v={r.get('VGPRs', '?'):>4} a={r.get('AGPRs', '?'):>4} "
              f"spill={r.get('VGPRs Spill', '?'):>4} occ={r.get('Occupancy [waves/SIMD]', '?')}")
