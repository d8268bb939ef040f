"""Times the device generator (rsl_synth_cube) for 1000 cfg2 frames with hipEvents."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'radar-slam_amd'))
import torch  # noqa: E402
import rsl  # noqa: E402

ctx = rsl.get_context(0)
gen = rsl.SyntheticCubes(ctx, [dict(range_sc=20.0, rcs=-10.0)], chirp_duration=51.2e-6, num_chirps=128,
                         num_antennas=8, noise_power=0.01)
out = gen.generate(1000, seed=1)
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ms = []
for i in range(5):
    a.record()
    gen.generate(1000, seed=1, frame0=i * 1000, out=out)
    b.record()
    torch.cuda.synchronize()
    ms.append(a.elapsed_time(b))
gb = out.numel() * 8 / 1e9
print(f"rsl_synth_cube 1000 cfg2 frames: {min(ms):.3f} ms (min of 5), {gb / min(ms):.2f} TB/s written")
