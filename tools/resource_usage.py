"""Summarise hipcc -Rpass-analysis=kernel-resource-usage output (stdin) per kernel."""
import re
import subprocess
import sys

cur = None
rows = {}
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+(VGPRs|AGPRs|TotalSGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).split()[0]] = int(m.group(2))
for k, v in rows.items():
    name = re.sub(r"\(.*", "", k)[:110]
    print(f"{v.get('VGPRs',0):4d}v {v.get('TotalSGPRs',0):3d}s scr={v.get('ScratchSize',0):4d} occ={v.get('Occupancy',0)} lds={v.get('LDS',0):6d}  {name}")
