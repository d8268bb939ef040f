"""Register / spill / occupancy report of every kernel in one .hip file (hipcc -Rpass-analysis=kernel-resource-usage),
compiled with the Makefile's flags for that file.   python tools/regs.py radar-slam_amd/csrc/rsl_doa_toep.hip [filter] [--dev]"""
import re
import subprocess
import sys

src = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ''
dev = '--dev' in sys.argv[3:]  # the development build's variants (-DRSL_DEV_KNOBS)
flags = (['-DRSL_DEV_KNOBS'] if dev else []) + ['-O3', '-std=c++17', '--offload-arch=gfx950', '-Rpass-analysis=kernel-resource-usage', '-c', src, '-o',
         '/tmp/_regs.o']
if 'doa' in src:
    flags[:0] = ['-fno-slp-vectorize']
if 'doa_toep' in src:
    flags[:0] = ['-mllvm', '-amdgpu-mfma-vgpr-form=1']
out = subprocess.run(['/opt/rocm/bin/hipcc'] + flags, capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r'Function Name: (\S+)', line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r'remark:\s+([A-Za-z /\[\]]+?):\s+(\d+)', line)
    if m and cur:
        rows[cur][m.group(1).strip()] = int(m.group(2))
for name, r in rows.items():
    if filt in name:
        print(f"{r.get('VGPRs', '?'):4} vgpr {r.get('AGPRs', 0):3} agpr {r.get('VGPRs Spill', 0):3} spill "
              f"occ {r.get('Occupancy [waves/SIMD]', '?')}  {name[:110]}")
