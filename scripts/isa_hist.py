"""Instruction histogram of one kernel in a hipcc -S listing: python scripts/isa_hist.py file.s name-substring [N]"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
want = sys.argv[2]
n = int(sys.argv[3]) if len(sys.argv) > 3 else 40
names = [l.split(":")[0] for l in s.split("\n") if re.match(r"^[A-Za-z_][\w.]*:", l) and want in l.split(":")[0]]
name = names[0]
i = s.index(name + ":")
j = s.index(".Lfunc_end", i)
c = collections.Counter()
for l in s[i:j].split("\n"):
    l = l.strip()
    if not l or l.startswith((".", ";")) or l.endswith(":"):
        continue
    c[l.split()[0]] += 1
print(name)
for k, v in c.most_common(n):
    print(f"{v:6d} {k}")
