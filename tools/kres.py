"""Per-kernel VGPR / spill / occupancy table from ``hipcc -Rpass-analysis=kernel-resource-usage`` output.

    hipcc ... -Rpass-analysis=kernel-resource-usage 2>&1 | python tools/kres.py [substring]
"""
import re
import sys

cur, rows = None, []
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    if cur is None:
        continue
    for key, pat in (("vgpr", r" VGPRs: (\d+)"), ("spill", r"VGPRs Spill: (\d+)"), ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"),
                     ("lds", r"LDS Size \[bytes/block\]: (\d+)")):
        m = re.search(pat, line)
        if m:
            cur[key] = int(m.group(1))
sub = sys.argv[1] if len(sys.argv) > 1 else ""
for r in rows:
    if sub in r["name"]:
        print(f"{r.get('vgpr', '?'):>4} vgpr  spill {r.get('spill', '?'):>3}  occ {r.get('occ', '?')}  lds {r.get('lds', '?'):>6}  {r['name']}")
