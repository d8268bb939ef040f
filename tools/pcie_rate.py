"""PCIe-inclusive throughput of the cfg2 chain, standalone: bench.py's `pcie_inclusive` side measurement
(the metric's `value` starts with the cubes resident in HBM; this is the rate when every frame's c64 cube first
crosses PCIe from pinned host memory).

    python tools/pcie_rate.py [--frames 500] [--steps 8]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'radar-slam_amd'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--frames', type=int, default=500)
    ap.add_argument('--steps', type=int, default=8)
    args = ap.parse_args()
    import torch
    import rsl
    from bench import pcie_inclusive
    dev = torch.device('cuda', 0)
    print(json.dumps(pcie_inclusive(rsl.get_context(0), dev, args.frames, args.steps)))


if __name__ == '__main__':
    main()
