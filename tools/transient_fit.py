"""Which wrong operand explains the round-4 pipelined-mode K1 fault?  

Input: gpurun_out/transient_row.npz (tools/transient_row.py: the faulting chirp row's cube samples, the dechirp table
and the serial K1 output) and the recorded pipelined values (gpurun_out/r4c_diag_g1.log).  k_range_fft_p<256> runs the
256-point FFT as two radix-16 Stockham stages; stage-2 butterfly j (lane j of one 16-lane pass) reads
v[r] = Z[j + 16 r] W256^(r j), r < 16, and Dft<16> (rsl_common.h) writes X[j + 16 k].  The recorded error sits in
outputs k = 1, 5, 9, 13 of all 16 butterflies as delta_j (1 - i) with alternating sign, i.e. an error e_j = delta_j / h
(h = 1/sqrt 2) in the real part of y'[2][1] = (v2 - v10) + (-i)(v6 - v14), the value that the W16^2 product reads
(v110 in the ISA listing of DESIGN §4).  This script rebuilds every butterfly's inputs in fp64 from the cube row,
checks them against the serial K1 output, and scores candidate mechanisms: e_j equal, lane by lane, to the difference
between the right operand and some other register value (a stale value, the other half of a packed pair, a
neighbouring lane's value).  CPU:  python tools/transient_fit.py"""
import ast
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
d = np.load(os.path.join(ROOT, 'gpurun_out', 'transient_row.npz'))
x = d['cube'].astype(np.complex128) * d['table'].astype(np.complex128)
N, R = 256, 16
W = lambda k, n: np.exp(-2j * np.pi * k / n)
# stage 1: butterfly j1 reads x[j1 + 16 r], writes Z[16 j1 + k]
Z = np.zeros(N, complex)
for j1 in range(R):
    Z[16 * j1:16 * j1 + 16] = np.fft.fft(x[j1::16])
v = np.array([[Z[j + 16 * r] * W(r * j, N) for r in range(R)] for j in range(R)])  # v[j][r]: stage-2 inputs
X = np.zeros(N, complex)
for j in range(R):
    X[j::16] = np.fft.fft(v[j])
work = d['work'].astype(np.complex128)
err = np.abs(X[1:] - work[1:]).max() / np.abs(work).max()
print(f'rebuilt K1 row vs serial K1 output (bins 1..255): max rel err {err:.2e}')

# recorded pipelined values (bins 16..31 = output k = 1 of butterflies j = 0..15)
log = open(os.path.join(ROOT, 'gpurun_out', 'r4c_diag_g1.log')).read()
a = log.index('[index, serial, pipelined]: ') + len('[index, serial, pipelined]: ')
vals = ast.literal_eval(log[a:log.index(']; batch', a) + 1])
rec = {tuple(i)[3]: (s, p) for i, s, p in vals}
h = 0.70710678118654752440
e_obs = np.array([(rec[16 + j][1] - rec[16 + j][0]).real / h for j in range(R)])
chk = [max(abs((rec[k * 16 + j][1] - rec[k * 16 + j][0]) - s * h * e_obs[j] * (1 - 1j)) for j in range(R))
       for k, s in ((1, 1), (5, -1), (9, 1), (13, -1))]
print('error pattern delta_j (1 - i), sign + - + - over k = 1, 5, 9, 13: max deviation', max(chk))
print('e_j =', np.array2string(e_obs, precision=4))

# register values of Dft<16> in butterfly j (the packed pairs of the ISA listing), and candidate wrong operands
def regs(j):
    a = v[j]
    r = {}
    for n2 in range(4):
        t = [a[n2], a[4 + n2], a[8 + n2], a[12 + n2]]
        r[f't0_{n2}'] = t[0] + t[2]
        r[f't1_{n2}'] = t[0] - t[2]
        r[f't2_{n2}'] = t[1] + t[3]
        r[f'd_{n2}'] = t[1] - t[3]
        r[f'y{n2}1'] = (t[0] - t[2]) - 1j * (t[1] - t[3])
        r[f'y{n2}3'] = (t[0] - t[2]) + 1j * (t[1] - t[3])
    for n in range(16):
        r[f'v{n}'] = a[n]
    out = {}
    for k, c in r.items():
        out[k + '.x'] = c.real
        out[k + '.y'] = c.imag
    return out

rg = [regs(j) for j in range(R)]
right = np.array([rg[j]['y21.x'] for j in range(R)])
cands = []
for name in rg[0]:
    for lane_map, lname in ((lambda j: j, 'same lane'), (lambda j: j ^ 1, 'lane^1'), (lambda j: (j + 1) % 16, 'lane+1'),
                            (lambda j: (j - 1) % 16, 'lane-1'), (lambda j: j ^ 8, 'lane^8')):
        wrong = np.array([rg[lane_map(j)][name] for j in range(R)])
        for sgn in (1, -1):
            pred = sgn * wrong - right  # y21.x replaced by +-(that value)
            rel = np.abs(pred - e_obs).max() / np.abs(e_obs).max()
            cands.append((rel, f'y21.x <- {"-" if sgn < 0 else ""}{name} ({lname})'))
    # an operand of y21.x = t1_2.x + d_2.y replaced: e = wrong - right operand
    for op in ('t1_2.x', 'd_2.y'):
        for lane_map, lname in ((lambda j: j, 'same lane'), (lambda j: j ^ 1, 'lane^1')):
            wrong = np.array([rg[lane_map(j)][name] for j in range(R)])
            opv = np.array([rg[j][op] for j in range(R)])
            pred = wrong - opv
            rel = np.abs(pred - e_obs).max() / np.abs(e_obs).max()
            cands.append((rel, f'operand {op} <- {name} ({lname})'))
cands.sort()
print('best candidate mechanisms (max relative misfit over the 16 lanes):')
for rel, what in cands[:12]:
    print(f'  {rel:.3e}  {what}')
