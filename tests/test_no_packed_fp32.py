"""Guard for the pipelined-transient avoidance: no packed-FP32 VALU
(v_pk_add_f32 / v_pk_mul_f32 / v_pk_fma_f32) in any kernel that runs in the pipelined chain step -- K1 / K2 (range and
Doppler FFT + detection), detect / offsets / emit, the DoA scan and its fixup, the cell extras, velocity and the
trajectory kernels.  Both recorded wrong-result events of rounds 3 and 4 sat in a packed-FP32 instruction of a kernel
co-running with the MFMA scan; rsl_fft.hip compiles its kernels with target("no-packed-fp32-ops") and the other
pipelined kernels carry none either.  A compiler update or a new kernel outside the pragma would silently reopen it:
this test disassembles the gfx950 code objects of the built librsl.so and fails on any such instruction there.

The detector itself is pinned on a small kernel compiled here twice: with packed float2 arithmetic it must find
v_pk_* instructions, and with the same pragma as rsl_fft.hip it must find none.
"""
import os
import re
import shutil
import struct
import subprocess
from collections import Counter

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, 'radar-slam_amd', 'lib', 'librsl.so')
LLVM = '/opt/rocm/llvm/bin'
HIPCC = '/opt/rocm/bin/hipcc'
PK = re.compile(r'\bv_pk_(add|mul|fma)_f32\b')
# kernels of the pipelined step (bench.py step_pipelined: run_front / run_back / the trajectory step)
GUARDED = ('k_range_fft', 'k_doppler', 'k_range_dft', 'k_detect', 'k_offsets', 'k_emit', 'k_doa', 'k_cell_extras',
           'k_velocity', 'k_traj')
# kernels that must be found in the library, so that a renamed kernel cannot escape the guard unnoticed
MUST_SEE = ('k_range_fft_r512', 'k_doppler_detect_r128', 'k_range_fft_r1024', 'k_doppler_detect_r256', 'k_doa_toep',
            'k_doa_fixup', 'k_emit', 'k_velocity', 'k_traj_scan')

needs_tools = pytest.mark.skipif(not (os.path.exists(os.path.join(LLVM, 'llvm-objdump')) and
                                      os.path.exists(os.path.join(LLVM, 'llvm-objcopy'))),
                                 reason='ROCm llvm tools absent')


def gfx950_code_objects(path, tmp):
    """The gfx950 code objects of a host ELF: its .hip_fatbin section is a sequence of clang offload bundles
    ('__CLANG_OFFLOAD_BUNDLE__', entry count, then (offset, size, id length, id) per entry, offsets from the bundle
    start), one per translation unit with device code."""
    fb = os.path.join(tmp, 'fatbin.bin')
    subprocess.run([os.path.join(LLVM, 'llvm-objcopy'), f'--dump-section=.hip_fatbin={fb}', path,
                    os.path.join(tmp, 'stripped.so')], check=True, capture_output=True)
    d = open(fb, 'rb').read()
    magic = b'__CLANG_OFFLOAD_BUNDLE__'
    out, pos = [], 0
    while True:
        i = d.find(magic, pos)
        if i < 0:
            break
        n = struct.unpack_from('<Q', d, i + len(magic))[0]
        p = i + len(magic) + 8
        for _ in range(n):
            off, size, idl = struct.unpack_from('<QQQ', d, p)
            p += 24
            ident = d[p:p + idl].decode()
            p += idl
            if 'gfx950' in ident:
                out.append(d[i + off:i + off + size])
        pos = i + len(magic)
    return out


def packed_fp32_by_function(code_object, tmp, tag):
    """{demangled function name: count of packed-FP32 VALU instructions} (every function listed, 0 included)."""
    p = os.path.join(tmp, f'{tag}.co')
    open(p, 'wb').write(code_object)
    dis = subprocess.run([os.path.join(LLVM, 'llvm-objdump'), '-d', '--demangle', p], check=True,
                         capture_output=True, text=True).stdout
    cnt, cur = Counter(), None
    for line in dis.splitlines():
        m = re.match(r'^[0-9a-f]+ <(.*)>:$', line)
        if m:
            cur = m.group(1)
            cnt[cur] += 0
        elif cur is not None and PK.search(line):
            cnt[cur] += 1
    return cnt


@needs_tools
@pytest.mark.skipif(not os.path.exists(LIB), reason='librsl.so not built')
def test_pipelined_kernels_have_no_packed_fp32(tmp_path):
    objs = gfx950_code_objects(LIB, str(tmp_path))
    assert objs, 'no gfx950 code object in librsl.so'
    funcs = Counter()
    for j, co in enumerate(objs):
        funcs.update(packed_fp32_by_function(co, str(tmp_path), f'co{j}'))
    names = list(funcs)
    for k in MUST_SEE:
        assert any(re.search(rf'\brsl::{k}\b', n) for n in names), f'kernel {k} not found in librsl.so'
    bad = {n: c for n, c in funcs.items() if c and any(re.search(rf'\brsl::{g}', n) for g in GUARDED)}
    assert not bad, f'packed-FP32 VALU in pipelined-step kernels: {bad}'


SNIPPET = r'''
#include <hip/hip_runtime.h>
typedef float f2 __attribute__((ext_vector_type(2)));
%s
__global__ void k_probe(const f2* a, const f2* b, f2* o, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) o[i] = a[i] * b[i] + a[i];
}
%s
'''
PRAGMA = ('#if defined(__HIP_DEVICE_COMPILE__)\n'
          '#pragma clang attribute push(__attribute__((target("no-packed-fp32-ops"))), apply_to = function)\n#endif',
          '#if defined(__HIP_DEVICE_COMPILE__)\n#pragma clang attribute pop\n#endif')


@needs_tools
@pytest.mark.skipif(not os.path.exists(HIPCC) or shutil.which(HIPCC) is None, reason='hipcc absent')
def test_detector_sees_packed_fp32_and_pragma_removes_it(tmp_path):
    counts = []
    for with_pragma in (False, True):
        src = tmp_path / f'probe{int(with_pragma)}.hip'
        src.write_text(SNIPPET % (PRAGMA if with_pragma else ('', '')))
        so = tmp_path / f'probe{int(with_pragma)}.so'
        subprocess.run([HIPCC, '-O3', '-fPIC', '-shared', '--offload-arch=gfx950', str(src), '-o', str(so)],
                       check=True, capture_output=True)
        objs = gfx950_code_objects(str(so), str(tmp_path))
        c = Counter()
        for j, co in enumerate(objs):
            c.update(packed_fp32_by_function(co, str(tmp_path), f'p{int(with_pragma)}_{j}'))
        counts.append(sum(v for n, v in c.items() if 'k_probe' in n))
    assert counts[0] > 0, 'the probe kernel compiled without the pragma shows no packed FP32: the detector is blind'
    assert counts[1] == 0, 'the pragma no longer removes packed FP32'
