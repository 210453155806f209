"""Tabulate hipcc -Rpass-analysis=kernel-resource-usage remarks: kernel, VGPRs, SGPRs, spills, occupancy.
usage: usage_table.py build/kern_u8.usage [NAME_SUBSTRING]"""
import re
import sys

cur, rows = None, []
for line in open(sys.argv[1]):
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[bytes/lane\])?: (\S+)", line)
    if m and cur is not None:
        cur[m.group(1).strip()] = m.group(2)
flt = sys.argv[2] if len(sys.argv) > 2 else ""
for r in rows:
    if flt in r["name"]:
        print(f"{r['name'][:60]:60s} vgpr {r.get('VGPRs', '?'):>4} sgpr {r.get('TotalSGPRs', '?'):>4} "
              f"vspill {r.get('VGPRs Spill', '?'):>3} sspill {r.get('SGPRs Spill', '?'):>3} "
              f"scratch {r.get('ScratchSize', '?'):>3} occ {r.get('Occupancy [waves/SIMD]', '?')}")
