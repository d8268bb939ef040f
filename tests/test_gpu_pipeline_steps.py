"""GPU: the file-staged steps of the reference's drop-in caller, scripts/run_ego_motion_pipeline.py,
restated call for call on the build's src.* modules and checked against the oracle.

  step 2 (:134-181)  SignalPreprocessor(**params) per frame .npy -> process_frame: *_rds.npy + *_rds_peaks.npz
  step 3 (:183-232)  extract_angles_from_rds(method='music') -> *_angles.npz (targets pickled)
  step 4 (:234-289)  estimate_velocity_from_angles keeps the reference's ``targets.item()`` on the loaded object array
                     (velocity_solver.py:438): ValueError for more than one target
  (step 5's PoseIntegrator is covered by tests/test_gpu_traj.py and tests/test_gpu_dropin.py)
The files are the build's own outputs (loaded with allow_pickle as the reference's wrappers do).
"""
import glob
import os

import numpy as np
import pytest

import parity as P
import radar_oracle as O

pytestmark = pytest.mark.gpu

A, C, TC = 8, 32, 12.8e-6  # S = 128
PARAMS = dict(fc=77e9, bandwidth=1e9, chirp_duration=TC, pri=100e-6, num_chirps=C, sampling_rate=10e6)


@pytest.fixture(scope='module')
def staged(tmp_path_factory, ctx):
    d = tmp_path_factory.mktemp('pipeline')
    for k in ('raw_sim', 'rds', 'angles', 'velocities', 'poses'):
        (d / k).mkdir()
    frames = []
    for f in range(2):  # step 1's output: frame_XXXX.npy, complex128 [A, C, S] (simulate_raw.py:147-221)
        np.random.seed(1000 + f)
        fr = O.synthesize_frame(O.TEST_SCENE, chirp_duration=TC, num_chirps=C, num_antennas=A)
        np.save(d / 'raw_sim' / f'frame_{f:04d}.npy', fr)
        frames.append(fr)
    return d, frames


def test_step2_process_frame(staged):
    from src.radar_signal.dechirp import process_frame
    d, frames = staged
    for f, path in enumerate(sorted(glob.glob(str(d / 'raw_sim' / 'frame_*.npy')))):
        out = str(d / 'rds' / (os.path.basename(path).replace('.npy', '_rds.npy')))
        res = process_frame(path, out, PARAMS)
        rds = np.load(out)
        assert rds.dtype == np.complex128 and rds.shape == (A, 128, C) and res['rds_shape'] == rds.shape
        ref = O.range_doppler_spectrum(frames[f], chirp_duration=TC)
        assert P.rds_error(rds, ref) <= P.RDS_ATOL_REL
        pk = dict(np.load(out.replace('.npy', '_peaks.npz'), allow_pickle=True))
        assert set(pk) == {'peaks', 'range_bins_m', 'doppler_bins_hz', 'power_spectrum_db'}
        assert len(pk['peaks']) == res['num_peaks']
        refp = O.extract_peaks(ref)['peaks']
        key = lambda ps: {(int(p['antenna']), int(p['range_bin']), int(p['doppler_bin'])) for p in ps}
        assert len(key(pk['peaks']) ^ key(refp)) <= 2  # near-tie decisions only (tests/parity.py)


def test_step3_extract_angles(staged):
    from src.angle_estimation.angle_estimation import extract_angles_from_rds
    d, frames = staged
    for rds_path in sorted(glob.glob(str(d / 'rds' / '*_rds.npy'))):
        out = str(d / 'angles' / os.path.basename(rds_path).replace('_rds.npy', '_angles.npz'))
        res = extract_angles_from_rds(rds_path, rds_path.replace('.npy', '_peaks.npz'), out, method='music')
        z = np.load(out, allow_pickle=True)
        targets = list(z['targets'])
        assert len(targets) == res['num_targets'] > 0
        rds = np.load(rds_path)
        sigs = np.array([O.spatial_signature(rds, int(t['range_bin']), int(t['doppler_bin'])) for t in targets])
        grid = O.azimuth_grid()
        idx = np.array([int(np.argmin(np.abs(grid - t['azimuth_deg']))) for t in targets])
        nm, nu, _ = P.doa_diff(idx, sigs, O.steering_matrix(grid, A), 'music')
        assert nu == 0 and nm <= P.doa_flip_budget(len(targets)), (nm, nu)


def test_step4_velocity_quirk(staged):
    from src.velocity_solver.velocity_solver import estimate_velocity_from_angles
    d, _ = staged
    ang = sorted(glob.glob(str(d / 'angles' / '*_angles.npz')))
    rds = sorted(glob.glob(str(d / 'rds' / '*_rds.npy')))
    assert ang and rds
    with pytest.raises(ValueError):  # more than one target: .item() on the object array (velocity_solver.py:438)
        estimate_velocity_from_angles(ang[0], rds[0], str(d / 'velocities' / 'v.npz'))

