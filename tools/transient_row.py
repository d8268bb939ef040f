"""Inputs of the round-4 pipelined-mode wrong result (gpurun_out/r4c_diag_g1.log: K1 `work` of batch 1, frame 0,
antenna 4, chirp 15 differed from the serial run at range bins 16-31, 80-95, 144-159, 208-223).  Regenerates the same
seeded cubes as tests/test_gpu_pipelined.py (_cubes: torch's device generator, seed 11) and runs the serial chain once,
then saves that chirp's cube row, the dechirp table and the serial K1 output row, so that tools/transient_fit.py can
rebuild the stage-2 DFT16 inputs of every butterfly on the CPU and test which wrong operand explains the recorded
pipelined values.  GPU box:  python tools/transient_row.py  ->  gpurun_out/transient_row.npz"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'radar-slam_amd'), ROOT, os.path.join(ROOT, 'tests')]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import rsl  # noqa: E402
import test_gpu_pipelined as T  # noqa: E402

ctx = rsl.get_context(0)
cfg = rsl.ChainConfig(num_antennas=T.A, num_chirps=T.C, chirp_duration=T.TC)
cubes = T._cubes()
ch = rsl.RadarChain(cfg, T.F, ctx)
ch.run(cubes[1])
torch.cuda.synchronize()
os.makedirs(os.path.join(ROOT, 'gpurun_out'), exist_ok=True)
np.savez(os.path.join(ROOT, 'gpurun_out', 'transient_row.npz'),
         cube=cubes[1][0, 4, 15].cpu().numpy(), table=ch.table.cpu().numpy(), work=ch.work[0, 4, 15].cpu().numpy(),
         work_c14=ch.work[0, 4, 14].cpu().numpy())
print('saved', flush=True)
