"""FFT stage (K1 + K2) over one 2000-frame cfg2 batch: one launch pair vs chunks of N frames on two alternating
streams (own handle and chunk-sized `work` per stream), with the packed `work` stored non-temporally (product) or
temporally (dev library, RSL_WORK_TEMPORAL=1: may stay in the 256 MiB Infinity Cache until the chunk's K2 reads it).
Round 3's tools/archive/chunk_mall.py measured only the nt form (5.63 vs 5.24 ms at N = 32).  Outputs must be
bit-identical to the one-launch run.
GPU box:  RSL_LIBRARY=radar-slam_amd/lib/librsl_dev.so [RSL_WORK_TEMPORAL=1] python tools/chunk_mall2.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'radar-slam_amd'), ROOT, os.path.join(ROOT, 'tools', 'archive')]
os.environ.setdefault('CHUNKS', '16,32,48,64,100')
import chunk_mall as M  # noqa: E402  (the round-3 harness: one / chunked / timed, then prints its table)
