"""HBM copy rate on this box (torch's copy kernel, read + write), the practical ceiling the streaming kernels are
compared against:  python tools/copy_rate.py"""
import torch

n = 1 << 30  # 8 GiB per c64 buffer
a = torch.empty(n, dtype=torch.complex64, device='cuda')
b = torch.empty_like(a)
a.real.fill_(1.0)
for _ in range(2):
    b.copy_(a)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(5):
    b.copy_(a)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 5
print(f'copy {2 * n * 8 / 1e9:.2f} GB in {ms:.3f} ms: {2 * n * 8 / ms / 1e9:.2f} TB/s')
