"""Parity at the batch sizes the bench times: one 2000-frame configs[2] batch and one
400-frame configs[4]-shape batch through rsl.RadarChain, on the bench's own device-synthesised cubes (bench.py
make_cubes: the reference simulator's scene, simulate_raw.py:102-221, plus Philox noise).

At these sizes the element indices reach 1.05e9 (cfg2: 2000 x 8 x 128 x 512) and 1.68e9 (cfg5: 400 x 16 x 256 x 1024)
per buffer, near 2^31, and the DoA scan runs on 32-bit cell indices.  For frames 0, F/2 and F-1 every output of the
batch must equal, bit for bit, a one-frame run of the same cube: RDS, masks, row counts, the frame's slice of the entry
and cell lists (packed coordinates, peak dB, the cell index relative to the frame's base, range-Doppler cell, antenna
mask), grid index, ESPRIT, phase and the velocity row.  Frame F/2 is also checked against the oracle (RDS, peak set,
MUSIC argmax rule, ESPRIT, the LS velocity at the GPU's own angles), and the batch's entry and cell totals against the
list capacities.  Reference: dechirp.py:246-271 (order-preserving peak list)."""
import os
import sys

import numpy as np
import pytest
import torch

import parity as P
import radar_oracle as O

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SHAPES = {'cfg2': (8, 128, 51.2e-6, 2000), 'cfg5': (16, 256, 102.4e-6, 400)}
DOA_SAMPLE = 20000


def _bits(t):
    t = t.contiguous()
    if t.is_complex():
        t = t.view(torch.float32)
    if t.dtype == torch.float32:
        return t.view(torch.int32)
    if t.dtype == torch.float64:
        return t.view(torch.int64)
    return t


def _frame_outputs(ch, f, cb, eb):
    """Frame f's outputs of a chain (device tensors), list indices made frame-relative."""
    L = ch.lists
    es, cs = slice(int(eb[f]), int(eb[f + 1])), slice(int(cb[f]), int(cb[f + 1]))
    return {'rds': ch.rds[f], 'mask': ch.mask[f], 'row_count': ch.row_count[f],
            'e_coord': L['e_coord'][es], 'e_pdb': L['e_pdb'][es], 'e_cell': L['e_cell'][es] - int(cb[f]),
            'c_rc': L['c_rc'][cs], 'c_amask': L['c_amask'][cs], 'c_frame': L['c_frame'][cs] - f,
            'gidx': ch.gidx[cs], 'esprit': ch.ext['esprit'][cs], 'phase': ch.ext['phase'][cs], 'vel': ch.vel[f]}


@pytest.mark.parametrize('name', list(SHAPES))
def test_bench_batch_matches_single_frames(ctx, name):
    sys.path.insert(0, ROOT)
    import bench
    import rsl
    A, C, Tc, F = SHAPES[name]
    cfg = rsl.ChainConfig(num_antennas=A, num_chirps=C, chirp_duration=Tc, ridge=0.01)
    cube = bench.make_cubes(ctx, 1, F, A, C, Tc, 0)[0]
    big = rsl.RadarChain(cfg, F, ctx)
    big.run(cube)
    torch.cuda.synchronize()
    ne, nc = big.totals()
    assert 0 < ne <= big.entry_cap and 0 < nc <= big.cell_cap, (ne, big.entry_cap, nc, big.cell_cap)
    cb = big.offs['cell_base'].cpu().numpy()
    eb = big.offs['entry_base'].cpu().numpy()
    assert cb[0] == 0 and eb[0] == 0 and (np.diff(cb) >= 0).all() and (np.diff(eb) >= 0).all()
    assert cb[F] == nc and eb[F] == ne
    one = rsl.RadarChain(cfg, 1, ctx)
    frames = (0, F // 2, F - 1)
    for f in frames:
        one.run(cube[f:f + 1])
        torch.cuda.synchronize()
        cb1 = one.offs['cell_base'].cpu().numpy()
        eb1 = one.offs['entry_base'].cpu().numpy()
        assert eb1[1] == eb[f + 1] - eb[f] and cb1[1] == cb[f + 1] - cb[f], (f, eb1, cb1)
        got, ref = _frame_outputs(big, f, cb, eb), _frame_outputs(one, 0, cb1, eb1)
        for k in got:
            assert torch.equal(_bits(got[k]), _bits(ref[k])), f'{name}: frame {f} of the {F}-frame batch: {k} differs'
    # frame F/2 against the oracle
    f = F // 2
    frame = cube[f].cpu().numpy().astype(np.complex128)
    rds_ref = O.range_doppler_spectrum(frame, chirp_duration=Tc)
    rds = big.rds[f].cpu().numpy()
    err = P.rds_error(rds, rds_ref)
    assert err <= P.RDS_ATOL_REL, (name, err)
    W = big.mask.shape[-1]
    words = big.mask[f].cpu().numpy()
    bits = np.unpackbits(words.view(np.uint8).reshape(A, -1, W, 8), axis=-1, bitorder='little')
    gm = bits.reshape(A, -1, W * 64)[:, :, :C].astype(bool)
    ng, nr, nd, nu = P.peak_diff(gm, rds_ref, gate=(big.i_lo, big.i_hi))
    assert nu == 0 and nd <= max(2, 1e-4 * nr), (name, ng, nr, nd, nu)
    cs = slice(int(cb[f]), int(cb[f + 1]))
    rc = big.lists['c_rc'][cs].cpu().numpy()
    gidx = big.gidx[cs].cpu().numpy()
    esp = big.ext['esprit'][cs].cpu().numpy()
    ph = big.ext['phase'][cs].cpu().numpy()
    amask = big.lists['c_amask'][cs].cpu().numpy()
    sel = np.arange(len(rc))
    if len(sel) > DOA_SAMPLE:
        sel = np.sort(np.random.RandomState(5).choice(sel, DOA_SAMPLE, replace=False))
    ii, jj = rc[sel] // C, rc[sel] % C
    steer = O.steering_matrix(O.azimuth_grid(), A)
    sigs = np.stack([O.spatial_signature(rds_ref, i, j) for i, j in zip(ii, jj)])
    stats = {}
    nm, nuq, _ = P.doa_diff(gidx[sel], sigs, steer, 'music', stats=stats)
    ns, _ = P.scan_flips(gidx[sel], rds[:, ii, jj].T, steer, 'music')
    assert ns == 0 and nuq == 0 and nm <= P.doa_flip_budget(len(sel), A), (name, nm, nuq, ns, stats)
    emax, nnan = P.esprit_diff(esp[sel], O.esprit_closed(sigs))
    assert nnan == 0 and emax <= P.ESPRIT_TOL_DEG, (name, emax)
    # the frame's LS velocity (ridge 0.01 on v_x, v_y) at the GPU's own angles and phases, every cell
    w = np.array([bin(int(m) & 0xffffffff).count('1') for m in amask])
    az = np.repeat(np.radians(big.grid[gidx]), w)
    y = np.repeat(ph, w)
    vx, vy, cost = O.velocity_ls(az, y, lambda_c=3e8 / cfg.fc, ridge=0.01)
    v = big.vel[f].cpu().numpy()
    assert abs(v[2] - cost) <= P.VEL_COST_RTOL * cost
    assert abs(v[0] - vx) < P.VEL_ATOL and abs(v[1] - vy) < P.VEL_ATOL
    assert int(v[5]) == len(y)
    print(f'\n{name}: F={F}, entries {ne}, cells {nc} (caps {big.entry_cap}, {big.cell_cap}); frames {frames} '
          f'bit-identical to one-frame runs; frame {f}: RDS err {err:.2e}, DoA flips {nm}/{len(sel)}')
