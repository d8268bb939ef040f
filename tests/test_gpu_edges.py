"""GPU edge cases of the batched chain (rsl.RadarChain over librsl): empty and peak-free frames inside a batch,
an empty batch, and capacity-sized peak / cell lists that overflow.

The reference handles one frame at a time, so these are properties of the batching, checked against the same
chain on the same cubes (bit-exact: per-frame results must not depend on what else is in the batch or on the
list capacity) and, for the velocity of a truncated list, against the oracle's LS solve (velocity_solver.py:178-355
restated in oracle/radar_oracle.py:velocity_ls).
"""
import numpy as np
import pytest

import parity as P
import radar_oracle as O

pytestmark = pytest.mark.gpu

A, C, TC = 8, 64, 25.6e-6  # cfg1 frame shape (S = 256)
KEYS_E = ('e_ant', 'e_rbin', 'e_dbin', 'e_cell', 'e_pdb')
KEYS_C = ('c_frame', 'c_rc', 'c_amask', 'gidx', 'esprit', 'phase')
RAW_E = ('e_coord', 'e_cell', 'e_pdb')  # the device entry lists (packed coordinates, include/rsl.h)


def _frames(seeds):
    out = []
    for s in seeds:
        if s is None:
            out.append(np.zeros((A, C, 256), np.complex128))
        else:
            np.random.seed(s)
            out.append(O.synthesize_frame(O.TEST_SCENE, chirp_duration=TC, num_chirps=C, num_antennas=A))
    return np.stack(out)


def _run(ctx, frames, **kw):
    import rsl
    cfg = rsl.ChainConfig(num_antennas=A, num_chirps=C, chirp_duration=TC, **kw)
    ch = rsl.RadarChain(cfg, len(frames), ctx)
    ch.run(ctx.to_dev(frames.astype(np.complex64)))
    return ch


def _frame_slices(r, f):
    eb, cb = r['entry_base'], r['cell_base']
    e = {k: r[k][eb[f]:eb[f + 1]] for k in KEYS_E}
    c = {k: r[k][cb[f]:cb[f + 1]] for k in KEYS_C}
    c['c_frame'] = c['c_frame'] * 0  # frame index differs between batches
    e['e_cell'] = e['e_cell'] - cb[f]  # entry -> cell links are global list positions
    return e, c


def test_empty_frame_inside_batch(ctx):
    """A zero cube (no peaks) between two noisy frames: empty segments, and the other frames' entries, cells,
    angles and velocities identical to a batch without it."""
    r3 = _run(ctx, _frames([1000, None, 1001])).results()
    r2 = _run(ctx, _frames([1000, 1001])).results()
    assert r3['entry_base'][2] == r3['entry_base'][1] and r3['cell_base'][2] == r3['cell_base'][1]
    for f3, f2 in ((0, 0), (2, 1)):
        e3, c3 = _frame_slices(r3, f3)
        e2, c2 = _frame_slices(r2, f2)
        assert len(e3['e_ant']) > 0 and len(c3['c_rc']) > 0
        for k in KEYS_E:
            assert np.array_equal(e3[k], e2[k]), k
        for k in KEYS_C:
            assert np.array_equal(c3[k], c2[k]), k
        assert np.array_equal(r3['velocity'][f3], r2['velocity'][f2])
    v = r3['velocity'][1]
    assert v[5] == 0 and v[2] == 0  # no targets: n = 0, cost 0 (the host maps n < 3 to the reference's failure)


def test_batch_without_peaks(ctx):
    """Threshold above every cell: all lists empty, the DoA / velocity launches see zero cells."""
    ch = _run(ctx, _frames([1000, 1001]), threshold_db=100.0)
    r = ch.results()
    assert (r['entry_base'] == 0).all() and (r['cell_base'] == 0).all()
    assert len(r['e_ant']) == 0 and len(r['gidx']) == 0
    assert (r['velocity'][:, 5] == 0).all()


def test_empty_batch(ctx):
    ch = _run(ctx, np.zeros((0, A, C, 256), np.complex128))
    r = ch.results()
    assert r['entry_base'].tolist() == [0] and r['cell_base'].tolist() == [0]
    assert len(r['gidx']) == 0 and r['velocity'].shape[0] == 0


def test_capacity_overflow_truncates_in_bounds(ctx):
    """Lists far smaller than the batch's peaks: the host sees the overflow, the device writes exactly the first
    `cap` entries / cells (a prefix of the full lists, nothing past the capacity), DoA / ESPRIT / phase run on that
    prefix only, and the velocity segments end at the capacity."""
    torch = ctx.torch
    frames = _frames([1000, 1001])
    full_ch = _run(ctx, frames)
    full = full_ch.results()
    raw_full = {k: t.cpu().numpy() for k, t in full_ch.lists.items()}
    ch = _run(ctx, frames, entry_frac=1e-4, cell_frac=1e-4)
    ecap, ccap = ch.entry_cap, ch.cell_cap
    assert full['entry_base'][1] > ecap and full['cell_base'][1] > ccap  # frame 0 alone overflows both lists
    # re-run with lists 1024 slots longer than the capacity, filled with a sentinel: nothing past cap is written
    SENT = -7
    for k, t in list(ch.lists.items()):
        ch.lists[k] = torch.full((t.shape[0] + 1024,), SENT, dtype=t.dtype, device=t.device)
    ch.gidx = torch.full((ccap + 1024,), SENT, dtype=ch.gidx.dtype, device=ch.gidx.device)
    for k, t in list(ch.ext.items()):
        ch.ext[k] = torch.full((t.shape[0] + 1024,), SENT, dtype=t.dtype, device=t.device)
    ch.run(ctx.to_dev(frames.astype(np.complex64)))
    torch.cuda.synchronize()
    with pytest.raises(RuntimeError, match='capacity exceeded'):
        ch.results()
    assert ch.totals() == (int(full['entry_base'][2]), int(full['cell_base'][2]))  # true counts still reported
    lists = {k: t.cpu().numpy() for k, t in ch.lists.items()}
    lists['gidx'] = ch.gidx.cpu().numpy()
    lists.update({k: t.cpu().numpy() for k, t in ch.ext.items() if k != 'az'})
    for k in RAW_E:
        assert np.array_equal(lists[k][:ecap], raw_full[k][:ecap]), k
        assert (lists[k][ecap:] == SENT).all(), k
    for k in KEYS_C:
        assert np.array_equal(lists[k][:ccap], full[k][:ccap]), k
        assert (lists[k][ccap:] == SENT).all(), k
    # velocity: frame 0 solved on the first ccap cells, frame 1's segment is empty
    vel = ch.vel.cpu().numpy()
    sl = slice(0, ccap)
    w = np.array([bin(int(m) & 0xffffffff).count('1') for m in full['c_amask'][sl]])
    az = np.repeat(np.radians(full['grid'][full['gidx'][sl]]), w)
    y = np.repeat(full['phase'][sl], w)
    vx, vy, cost = O.velocity_ls(az, y, lambda_c=3e8 / ch.cfg.fc)
    assert int(vel[0, 5]) == len(y)
    assert abs(vel[0, 2] - cost) <= P.VEL_COST_RTOL * max(cost, 1e-12)
    assert abs(vel[0, 0] - vx) < P.VEL_ATOL and abs(vel[0, 1] - vy) < P.VEL_ATOL
    assert vel[1, 5] == 0
