"""Debug helper: run the chain on small configs and dump intermediates to gpurun_out/dbg_<name>.npz."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'radar-slam_amd'), os.path.join(ROOT, 'oracle')]
import radar_oracle as O
import rsl

CFGS = {'tiny': (8, 16, 3.2e-6), 'cfg1': (8, 64, 25.6e-6), 'odd400': (8, 16, 40e-6)}
ctx = rsl.get_context(0)
os.makedirs(os.path.join(ROOT, 'gpurun_out'), exist_ok=True)
for name in sys.argv[1:] or list(CFGS):
    A, C, Tc = CFGS[name]
    F = 2
    frames = []
    for f in range(F):
        np.random.seed(1000 + f)
        frames.append(O.synthesize_frame(O.TEST_SCENE, chirp_duration=Tc, num_chirps=C, num_antennas=A))
    frames = np.stack(frames)
    cfg = rsl.ChainConfig(num_antennas=A, num_chirps=C, chirp_duration=Tc)
    ch = rsl.RadarChain(cfg, F, ctx)
    cube = ctx.to_dev(frames.astype(np.complex64))
    ch.run(cube)
    ctx.sync()
    d = dict(frames=frames, rds=ch.rds.cpu().numpy(), work=ch.work.cpu().numpy(), mask=ch.mask.cpu().numpy(),
             row_count=ch.row_count.cpu().numpy(), entry_base=ch.offs['entry_base'].cpu().numpy(),
             cell_base=ch.offs['cell_base'].cpu().numpy(), frame_counts=ch.offs['frame_counts'].cpu().numpy(),
             entry_row_off=ch.offs['entry_row_off'].cpu().numpy(), cell_row_off=ch.offs['cell_row_off'].cpu().numpy(),
             i_lo=ch.i_lo, i_hi=ch.i_hi)
    np.savez(os.path.join(ROOT, 'gpurun_out', f'dbg_{name}.npz'), **d)
    ref = O.range_doppler_spectrum(frames[0], chirp_duration=Tc)
    print(name, 'rds err', np.abs(d['rds'][0] - ref).max() / np.abs(ref).max(), 'counts', d['frame_counts'])
