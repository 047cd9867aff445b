"""Per-kernel register / spill / occupancy table of one HIP source (hipcc -Rpass-analysis).
usage: python tools/kres.py ctpa-clip_amd/csrc/peg.hip [name-filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ''
out = subprocess.run(['/opt/rocm/bin/hipcc', '--offload-arch=gfx950', '-O3', '-std=c++17', '-fPIC', '-c', src, '-o',
                      '/tmp/_kres.o', '-Rpass-analysis=kernel-resource-usage'], capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r'Function Name: (\S+)', line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r'remark:\s+([A-Za-z \[\]/]+?):\s+(\d+)', line)
    if m and cur:
        rows[cur][m.group(1).strip()] = int(m.group(2))
for name, r in rows.items():
    if flt in name:
        dn = subprocess.run(['c++filt', name], capture_output=True, text=True).stdout.strip()
        print(f"{dn[:90]:90s} vgpr {r.get('VGPRs', '?'):>4} agpr {r.get('AGPRs', '?'):>4} "
              f"spill {r.get('VGPRs Spill', '?'):>3} occ {r.get('Occupancy [waves/SIMD]', '?')}")
