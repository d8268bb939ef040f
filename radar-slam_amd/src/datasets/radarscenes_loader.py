"""RadarScenes sequence access for the configs[3] pattern (the data format on the input side of the path).

Drop-in for ``src/datasets/radarscenes_loader.py`` of the reference (``RadarScenesLoader`` :24-254): the methods the
ego-motion analyzer calls (``radarscenes_complete_analysis.py:114-163``), with the same signatures, column names and
return shapes.  Host pandas only: these run once per sequence and feed the device replay (``rsl.replay``).

``load_sequence_data`` reads ``data/<sequence>/radar_data.h5`` with h5py, which is imported when the method runs (the
reference imports it at module top, :11): in an environment without h5py this module still imports, and the method
raises ImportError.  Plotting and quality-report helpers of the reference (:256-470) are out of scope.
"""
from __future__ import annotations

import json
import logging
from pathlib import Path
from typing import Dict, List, Optional

import numpy as np
import pandas as pd

logger = logging.getLogger(__name__)


class RadarScenesLoader:
    def __init__(self, dataset_path: str):
        self.dataset_path = Path(dataset_path)
        self.sensors_info = self._load_sensors_info()
        self.sequence_info = self._load_sequence_info()
        logger.info(f"Initialized RadarScenes loader for: {dataset_path}")
        logger.info(f"Found {len(self.sequence_info)} sequences")

    def _load_sensors_info(self) -> Dict:
        with open(self.dataset_path / "data" / "sensors.json", 'r') as f:
            return json.load(f)

    def _load_sequence_info(self) -> Dict:
        with open(self.dataset_path / "data" / "sequences.json", 'r') as f:
            return json.load(f)

    def load_sequence_data(self, sequence_id: str) -> Dict:
        """radar_data.h5 ('radar_data', 'odometry' tables) + scenes.json of one sequence (:55-112)."""
        import h5py  # not installed in every environment; only this method needs it
        path = self.dataset_path / "data" / sequence_id
        if not path.exists():
            raise ValueError(f"Sequence {sequence_id} not found")
        with h5py.File(path / "radar_data.h5", 'r') as f:
            radar_data = f['radar_data'][:]
            odometry_data = f['odometry'][:]
        with open(path / "scenes.json", 'r') as f:
            scenes = json.load(f)
        cam = path / "camera"
        camera_files = list(cam.glob("*.jpg")) if cam.exists() else []
        radar_df = pd.DataFrame(radar_data)
        odometry_df = pd.DataFrame(odometry_data)
        radar_df['datetime'] = pd.to_datetime(radar_df['timestamp'], unit='us')
        odometry_df['datetime'] = pd.to_datetime(odometry_df['timestamp'], unit='us')
        first, last = scenes['first_timestamp'], scenes['last_timestamp']
        return {'sequence_id': sequence_id, 'radar_data': radar_df, 'odometry_data': odometry_df, 'scenes_data': scenes,
                'camera_files': camera_files, 'sensors_info': self.sensors_info,
                'metadata': {'first_timestamp': first, 'last_timestamp': last, 'duration_ms': last - first,
                             'category': scenes.get('category', 'unknown')}}

    def extract_radar_frames(self, sequence_data: Dict, frame_duration_ms: float = 100.0) -> List[Dict]:
        """Fixed windows [t, t + frame_duration_ms) from the first radar timestamp; empty windows are dropped and
        each kept window groups its rows by sensor in order of first appearance (:139-192)."""
        df = sequence_data['radar_data']
        ts = df['timestamp'].to_numpy()
        t0, t1 = ts.min(), ts.max()
        step = frame_duration_ms * 1000
        frames = []
        cur = t0
        while cur < t1:
            end = cur + step
            sel = df[(df['timestamp'] >= cur) & (df['timestamp'] < end)].copy()
            if len(sel) > 0:
                groups = {sid: sel[sel['sensor_id'] == sid] for sid in sel['sensor_id'].unique()}
                frames.append({'frame_id': len(frames), 'timestamp': cur, 'frame_end_time': end, 'sensor_data': groups,
                               'total_measurements': len(sel), 'sensors': list(groups.keys())})
            cur = end
        logger.info(f"Extracted {len(frames)} radar frames")
        return frames

    def get_odometry_at_time(self, sequence_data: Dict, timestamp: int) -> Optional[Dict]:
        """The nearest odometry record if it is within 1 s (:194-224)."""
        odo = sequence_data['odometry_data']
        d = np.abs(odo['timestamp'] - timestamp)
        i = d.idxmin()
        if d.iloc[i] < 1e6:
            rec = odo.iloc[i]
            return {'timestamp': rec['timestamp'], 'x': rec['x_seq'], 'y': rec['y_seq'], 'yaw': rec['yaw_seq'],
                    'vx': rec['vx'], 'yaw_rate': rec['yaw_rate']}
        return None

    def convert_radar_to_scatterers(self, frame_data: Dict, sensor_id: int) -> pd.DataFrame:
        """The simulator's scatterer columns of one sensor's rows (:226-254)."""
        if sensor_id not in frame_data['sensor_data']:
            return pd.DataFrame()
        s = frame_data['sensor_data'][sensor_id]
        return pd.DataFrame({k: s[k].values for k in ('range_sc', 'azimuth_sc', 'rcs', 'vr', 'x_cc', 'y_cc')})


def load_radarscenes_sequence(dataset_path: str, sequence_id: str) -> Dict:
    """Module helper (:397-410): the sequence data of one sequence."""
    return RadarScenesLoader(dataset_path).load_sequence_data(sequence_id)
