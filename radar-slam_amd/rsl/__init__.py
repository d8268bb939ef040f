"""rsl — MI355X-native radar signal chain runtime (HIP kernels in librsl.so, bound with ctypes).

    from rsl import get_context, RadarChain, ChainConfig

Layers: ``_lib`` (C ABI, include/rsl.h) -> ``runtime.Context`` (device buffers, streams, timing) ->
``chain.RadarChain`` (batched cube -> velocity pipeline).  The reference-compatible classes live in
the ``src`` package next to this one (``src.radar_signal.dechirp.SignalPreprocessor`` ...).
"""
from ._lib import LIB_PATH, load  # noqa: F401
from .runtime import Context, get_context, unpack_coord  # noqa: F401
from .chain import ChainConfig, RadarChain  # noqa: F401
from .traj import TrajectoryReducer  # noqa: F401
from .synth import SyntheticCubes  # noqa: F401
from . import tables  # noqa: F401

__all__ = ['Context', 'get_context', 'ChainConfig', 'RadarChain', 'TrajectoryReducer', 'SyntheticCubes', 'tables', 'load',
           'LIB_PATH']
