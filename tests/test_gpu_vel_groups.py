"""K8 (k_velocity) on the grid-index path, the form the chain uses: rsl_velocity with (gidx, az_table, phase, antenna
mask).  The kernel reads the cells once: max |residual| comes from per-grid-index phase extremes and the residual sum
of squares from the moments, with a per-cell second pass only for a near-perfect fit (or when residuals are
requested).  Checked here against a per-cell numpy restatement of velocity_solver.py:142-176, 283-284 (cost, rmse,
max residual) on frames with zero-weight cells, an empty frame, a NaN phase and an exact fit, and the outputs must
not depend on whether residuals / predictions are requested."""
import numpy as np
import pytest

import radar_oracle as O

pytestmark = pytest.mark.gpu

K = 4 * np.pi * 0.1 / (3e8 / 77e9)


def _frames(rs, G):
    grid = np.radians(np.linspace(-90.0, 90.0, G))
    frames = []
    for f, n in enumerate((5000, 0, 37, 3000, 2000, 900)):
        g = rs.randint(0, G, n).astype(np.int32)
        m = rs.randint(0, 256, n).astype(np.uint32)
        m[rs.rand(n) < 0.1] = 0  # weight 0: in neither the sums nor the max residual
        if f == 4:  # exact model phases: the moment form cancels, the per-cell pass must take over
            y = K * (1.7 * np.cos(grid[g]) - 0.4 * np.sin(grid[g]))
        else:
            y = rs.uniform(-np.pi, np.pi, n)
        if f == 5:
            y[17] = np.nan
            m[17] = 3
        frames.append((g, y, m))
    return grid, frames


def _ref(grid, g, y, m, v, ridge):
    w = np.array([bin(int(x)).count('1') for x in m], dtype=np.float64)
    r = y - K * (v[0] * np.cos(grid[g]) + v[1] * np.sin(grid[g]))
    r2 = float((w * r * r).sum())
    rm = np.abs(r[w > 0])
    rm = float(np.nanmax(rm)) if len(rm) and not np.isnan(rm).all() else 0.0
    n = w.sum()
    return r2 + ridge * (v[0] ** 2 + v[1] ** 2), (np.sqrt(r2 / n) if n > 0 else 0.0), rm, n


@pytest.mark.parametrize('ridge', [0.0, 0.01])
def test_velocity_grid_path(ridge):
    import torch
    import rsl
    ctx = rsl.get_context()
    rs = np.random.RandomState(5)
    G = 361
    grid, frames = _frames(rs, G)
    seg = np.concatenate([[0], np.cumsum([len(fr[0]) for fr in frames])]).astype(np.int64)
    g = np.concatenate([fr[0] for fr in frames])
    y = np.concatenate([fr[1] for fr in frames])
    m = np.concatenate([fr[2] for fr in frames])
    d = dict(gidx=ctx.to_dev(g), az_table=ctx.to_dev(grid), amask=ctx.to_dev(m.view(np.int32)))
    o1, _, _ = ctx.velocity(None, ctx.to_dev(y), ctx.to_dev(seg), k=K, ridge=ridge, **d)
    o2, res, pred = ctx.velocity(None, ctx.to_dev(y), ctx.to_dev(seg), k=K, ridge=ridge, want_resid=True, **d)
    torch.cuda.synchronize()
    o1, o2 = o1.cpu().numpy(), o2.cpu().numpy()
    assert np.array_equal(o1, o2, equal_nan=True)  # same outputs with or without the per-cell outputs
    res = res.cpu().numpy()
    for f, (gf, yf, mf) in enumerate(frames):
        v = o1[f]
        cost, rmse, rm, n = _ref(grid, gf, yf, mf, v, ridge)
        assert v[5] == n
        if f == 5:  # a NaN phase of weight > 0: the cost is NaN as in the reference, max |r| ignores it (fmax)
            assert np.isnan(v[2]) and np.isnan(v[3]) and abs(v[4] - rm) <= 1e-12 * max(1.0, rm)
            continue
        if f == 4:  # exact fit: residuals are rounding noise (~1e-13; ~1e-8 with the ridge's shrinkage)
            assert abs(v[2] - cost) <= 1e-18 and v[3] < 1e-6 and abs(v[3] - rmse) <= 1e-6 * rmse + 1e-12, \
                (v[2], cost, v[3], rmse)
        else:
            assert abs(v[2] - cost) <= 1e-9 * cost, (f, v[2], cost)
            assert abs(v[3] - rmse) <= 1e-9 * max(rmse, 1e-12), (f, v[3], rmse)
        assert abs(v[4] - rm) <= 1e-12 * max(1.0, rm), (f, v[4], rm)
        if len(gf) >= 3:  # the solve itself against the oracle's exact box-constrained LS
            w = np.array([bin(int(x)).count('1') for x in mf])
            ox, oy, oc = O.velocity_ls(np.repeat(grid[gf], w), np.repeat(yf, w), lambda_c=3e8 / 77e9, ridge=ridge)
            assert abs(v[0] - ox) < 1e-7 and abs(v[1] - oy) < 1e-7
        sl = slice(seg[f], seg[f + 1])
        r = yf - K * (v[0] * np.cos(grid[gf]) + v[1] * np.sin(grid[gf]))
        assert np.allclose(res[sl], r, rtol=0, atol=1e-10)
