"""Instruction mix of one kernel's ISA by section (pass prologue / MFMA tile loop / rest), for VALU budgeting.
python tools/isa_mix.py file.hip kernel_substring"""
import collections
import re
import subprocess
import sys

src, sub = sys.argv[1], sys.argv[2]
flags = ['-O3', '-std=c++17', '--offload-arch=gfx950', '--cuda-device-only', '-S', src, '-o', '/tmp/_mix.s']
if 'doa' in src:
    flags[:0] = ['-fno-slp-vectorize']
if 'toep' in src:
    flags[:0] = ['-mllvm', '-amdgpu-mfma-vgpr-form=1']
subprocess.run(['/opt/rocm/bin/hipcc'] + flags, capture_output=True)
s = open('/tmp/_mix.s').read()
names = [m.group(1) for m in re.finditer(r'^(_Z[^\s:]+):', s, re.M) if sub in m.group(1)]
name = names[0]
a = s.index(name + ':')
b = s.index('.Lfunc_end', a)
body = s[a:b].split('\n')
hdr = [i for i, l in enumerate(body) if 'Loop Header: Depth=1' in l]
mf = [i for i, l in enumerate(body) if 'v_mfma' in l]


def mix(lo, hi):
    c = collections.Counter()
    for l in body[lo:hi]:
        m = re.match(r'\s+([sv]_\w+|global_\w+|ds_\w+|scratch_\w+|buffer_\w+)', l)
        if m:
            c[m.group(1)] += 1
    return c


secs = [('prologue', hdr[0] if hdr else 0, mf[0] if mf else len(body)),
        ('tileloop', mf[0] if mf else 0, mf[-1] + 1 if mf else 0), ('rest', mf[-1] + 1 if mf else 0, len(body))]
print(name[:100])
for tag, lo, hi in secs:
    c = mix(lo, hi)
    v = sum(n for k, n in c.items() if k.startswith('v_') and 'mfma' not in k)
    print(f"{tag}: VALU {v} SALU {sum(n for k, n in c.items() if k.startswith('s_'))} "
          f"mem {sum(n for k, n in c.items() if k.startswith(('global', 'ds_', 'scratch', 'buffer')))}")
    print('   ', c.most_common(18))
