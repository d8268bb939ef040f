"""Advanced regularised ego-motion optimisation on MI355X.

Drop-in for ``src/algorithms/advanced_velocity_optimization.py`` of the reference
(``AdvancedVelocityOptimizer`` :24-524, ``optimize_velocity_advanced`` :527-564): same constructor, state
(velocity history, adaptive bounds), methods, return types and dict keys.

The reference minimises the wrapped-phase cost plus piecewise penalties (:153-223) with several
differential-evolution runs (seed 42; DE ignores the initial guess, so the runs are identical).  Here each run
is ``rsl_wrapped_search`` mode 1: projected Gauss-Newton in (v_x, v_y) from every point of a grid whose spacing is
half the wrap period, over the adaptive bounds (a heuristic dense sampling of the basins, checked by the DE-cost
tests, not a guarantee that every basin is entered), then the 6-D refinement of the
best basins and the run's initial guess, keeping the lowest cost (see velocity_solver_improved.py for the basin
structure).  The penalties are evaluated on the device with the reference's exact formulas.
Parity contract: cost <= the reference's DE cost for the same associations, bounds and previous motion.
"""
from __future__ import annotations

import logging
from typing import Dict, List, Optional

import numpy as np

from rsl import ops

logger = logging.getLogger(__name__)

SPACING = 0.5  # stage-1 grid spacing of rsl_wrapped_search, as a fraction of the wrap period 2 pi / k


def _grid_starts(lo, hi, k):
    h = SPACING * 2 * np.pi / k
    return int(max(1, np.ceil((hi[0] - lo[0]) / h)) * max(1, np.ceil((hi[1] - lo[1]) / h)))


class AdvancedVelocityOptimizer:
    """Reference constructor / attributes / methods (advanced_velocity_optimization.py:24-524)."""

    def __init__(self, fc: float = 77e9, lambda_c: float = None, num_antennas: int = 8,
                 antenna_spacing: float = None, max_velocity: float = 50.0, max_angular_velocity: float = 10.0,
                 regularization_weight: float = 0.01, num_optimization_runs: int = 3, use_parallel: bool = True):
        self.fc = fc
        self.c = 3e8
        self.lambda_c = lambda_c or (self.c / self.fc)
        self.num_antennas = num_antennas
        self.antenna_spacing = antenna_spacing or (self.lambda_c / 2)
        self.max_velocity = max_velocity
        self.max_angular_velocity = max_angular_velocity
        self.regularization_weight = regularization_weight
        self.num_optimization_runs = num_optimization_runs
        self.use_parallel = use_parallel
        self.antenna_positions = np.arange(self.num_antennas) * self.antenna_spacing
        self.velocity_history = []
        self.angular_velocity_history = []
        self.adaptive_bounds = self._initialize_adaptive_bounds()
        logger.info("Initialized advanced velocity optimizer:")
        logger.info(f"  Max velocity: {max_velocity} m/s")
        logger.info(f"  Max angular velocity: {max_angular_velocity} rad/s")
        logger.info(f"  Regularization weight: {regularization_weight}")
        logger.info(f"  Optimization runs: {num_optimization_runs}")
        logger.info(f"  Parallel processing: {use_parallel}")

    def _initialize_adaptive_bounds(self) -> Dict:
        return {'velocity_bounds': [(-self.max_velocity, self.max_velocity)] * 3,
                'angular_velocity_bounds': [(-self.max_angular_velocity, self.max_angular_velocity)] * 3,
                'acceleration_bounds': [(-20, 20)] * 3,
                'angular_acceleration_bounds': [(-5, 5)] * 3}

    def update_adaptive_bounds(self, current_velocity: np.ndarray, current_angular_velocity: np.ndarray,
                               dt: float = 0.1) -> None:
        """State update after each solve (:94-151), identical bookkeeping."""
        self.velocity_history.append(np.array(current_velocity, copy=True))
        self.angular_velocity_history.append(np.array(current_angular_velocity, copy=True))
        max_history = 10
        if len(self.velocity_history) > max_history:
            self.velocity_history = self.velocity_history[-max_history:]
            self.angular_velocity_history = self.angular_velocity_history[-max_history:]
        if len(self.velocity_history) >= 2:
            vel_changes = np.diff(self.velocity_history, axis=0)
            ang_vel_changes = np.diff(self.angular_velocity_history, axis=0)
            max_acceleration = np.max(np.abs(vel_changes) / dt) if dt > 0 else 20.0
            max_angular_acceleration = np.max(np.abs(ang_vel_changes) / dt) if dt > 0 else 5.0
            safety_factor = 2.0
            self.adaptive_bounds['acceleration_bounds'] = [
                (-max_acceleration * safety_factor, max_acceleration * safety_factor)] * 3
            self.adaptive_bounds['angular_acceleration_bounds'] = [
                (-max_angular_acceleration * safety_factor, max_angular_acceleration * safety_factor)] * 3
            current_speed = np.linalg.norm(current_velocity)
            if current_speed > 0:
                direction = current_velocity / current_speed
                velocity_expansion = min(10.0, current_speed * 0.5)
                for i in range(3):
                    if direction[i] > 0:
                        self.adaptive_bounds['velocity_bounds'][i] = (
                            -self.max_velocity, min(self.max_velocity, current_velocity[i] + velocity_expansion))
                    else:
                        self.adaptive_bounds['velocity_bounds'][i] = (
                            max(-self.max_velocity, current_velocity[i] - velocity_expansion), self.max_velocity)

    def _k(self, dt):
        return 4 * np.pi * dt / self.lambda_c

    def _penalty(self, motion_params, previous_motion):
        """Regularisation terms of :188-219 (scalar; the data term runs on the device)."""
        w = self.regularization_weight
        velocity, angular_velocity = motion_params[:3], motion_params[3:]
        r = 0.0
        vm = np.linalg.norm(velocity)
        if vm > self.max_velocity * 0.8:
            r += w * (vm - self.max_velocity * 0.8) ** 2
        wm = np.linalg.norm(angular_velocity)
        if wm > self.max_angular_velocity * 0.8:
            r += w * (wm - self.max_angular_velocity * 0.8) ** 2
        if previous_motion is not None:
            r += w * 0.1 * np.sum((motion_params - previous_motion) ** 2)
        if vm > 20 and wm > 5:
            r += w * 0.01 * (vm - 20) * (wm - 5)
        r += w * 10.0 * velocity[2] ** 2
        return r

    def compute_regularized_cost_function(self, motion_params: np.ndarray, target_positions: np.ndarray,
                                          target_angles: np.ndarray, observed_phases: np.ndarray, dt: float,
                                          previous_motion: Optional[np.ndarray] = None) -> float:
        x = np.asarray(motion_params, np.float64)
        base = ops.phase_model(target_positions, target_angles, x, self._k(dt), y=observed_phases, wrap=True)['cost']
        return base + self._penalty(x, previous_motion)

    def _compute_phase_difference_model(self, target_positions: np.ndarray, target_angles: np.ndarray,
                                        velocity: np.ndarray, angular_velocity: np.ndarray, dt: float) -> np.ndarray:
        x = np.concatenate([np.asarray(velocity, np.float64).reshape(3),
                            np.asarray(angular_velocity, np.float64).reshape(3)])
        return ops.phase_model(target_positions, target_angles, x, self._k(dt))['pred']

    def generate_multiple_initial_guesses(self, target_associations: List[Dict], dt: float) -> List[np.ndarray]:
        guesses = [self._generate_smart_initial_guess(target_associations, dt), np.zeros(6)]
        for _ in range(self.num_optimization_runs - 2):  # global np.random, as the reference (:283-292)
            guesses.append(np.array([
                np.random.uniform(-self.max_velocity * 0.5, self.max_velocity * 0.5),
                np.random.uniform(-self.max_velocity * 0.5, self.max_velocity * 0.5),
                np.random.uniform(-5, 5),
                np.random.uniform(-self.max_angular_velocity * 0.5, self.max_angular_velocity * 0.5),
                np.random.uniform(-self.max_angular_velocity * 0.5, self.max_angular_velocity * 0.5),
                np.random.uniform(-self.max_angular_velocity * 0.5, self.max_angular_velocity * 0.5)]))
        return guesses

    def _generate_smart_initial_guess(self, target_associations: List[Dict], dt: float) -> np.ndarray:
        if not target_associations:
            return np.zeros(6)
        xy = lambda t: [t['range_m'] * np.cos(t['azimuth_rad']), t['range_m'] * np.sin(t['azimuth_rad']), 0]
        tv = np.array([(np.array(xy(a['current'])) - np.array(xy(a['previous']))) / dt for a in target_associations])
        med = np.median(tv, axis=0)
        return np.concatenate([np.append(-med[:2], 0), np.array([0, 0, 0])])

    def run_single_optimization(self, initial_guess: np.ndarray, target_positions: np.ndarray,
                                target_angles: np.ndarray, observed_phases: np.ndarray, dt: float,
                                previous_motion: Optional[np.ndarray] = None) -> Dict:
        bounds = self.adaptive_bounds['velocity_bounds'] + self.adaptive_bounds['angular_velocity_bounds']
        lo = [b[0] for b in bounds]
        hi = [b[1] for b in bounds]
        try:
            x, cost = ops.wrapped_search(target_positions, target_angles, observed_phases, self._k(dt), mode=1,
                                         lo=lo, hi=hi, nv=6, w=self.regularization_weight, vmax=self.max_velocity,
                                         wmax=self.max_angular_velocity, prev=previous_motion,
                                         extra=np.asarray(initial_guess, np.float64)[None], spacing_frac=SPACING)
            return {'success': True, 'motion_params': x, 'cost': cost, 'iterations': _grid_starts(lo, hi, self._k(dt)),
                    'initial_guess': initial_guess}
        except Exception as e:  # the reference reports a failed run and continues (:400-408)
            return {'success': False, 'motion_params': initial_guess, 'cost': float('inf'), 'iterations': 0,
                    'initial_guess': initial_guess, 'error': str(e)}

    def run_robust_optimization(self, target_associations: List[Dict], dt: float,
                                previous_motion: Optional[np.ndarray] = None) -> Dict:
        if len(target_associations) < 3:
            logger.warning("Insufficient target associations for optimization")
            return {'success': False, 'message': 'Insufficient target associations'}
        r = np.array([a['current']['range_m'] for a in target_associations], np.float64)
        az = np.array([a['current']['azimuth_rad'] for a in target_associations], np.float64)
        el = np.zeros_like(az)
        pos = np.stack([r * np.cos(el) * np.cos(az), r * np.cos(el) * np.sin(az), r * np.sin(el)], axis=1)
        ang = np.stack([az, el], axis=1)
        observed = np.array([a['temporal_phase_diff'] for a in target_associations])
        guesses = self.generate_multiple_initial_guesses(target_associations, dt)
        # runs are sequential device launches (the reference's ThreadPoolExecutor is GIL-bound, :457-469)
        results = [self.run_single_optimization(g, pos, ang, observed, dt, previous_motion) for g in guesses]
        ok = [x for x in results if x['success']]
        if not ok:
            logger.warning("All optimization runs failed")
            return {'success': False, 'message': 'All optimization runs failed'}
        best = min(ok, key=lambda x: x['cost'])
        motion = best['motion_params']
        velocity, angular_velocity = motion[:3], motion[3:]
        m = ops.phase_model(pos, ang, motion, self._k(dt), y=observed, wrap=True)
        predicted, residuals = m['pred'], m['resid']
        self.update_adaptive_bounds(velocity, angular_velocity, dt)
        return {'success': True, 'velocity': velocity, 'angular_velocity': angular_velocity, 'cost': best['cost'],
                'rmse': np.sqrt(np.mean(residuals ** 2)), 'max_residual': np.max(np.abs(residuals)),
                'residuals': residuals, 'predicted_phases': predicted, 'observed_phases': observed,
                'num_associations': len(target_associations), 'num_optimization_runs': len(results),
                'successful_runs': len(ok), 'best_initial_guess': best['initial_guess'], 'all_results': results}


def optimize_velocity_advanced(target_associations: List[Dict], dt: float = 0.1, radar_params: Dict = None,
                               previous_motion: Optional[np.ndarray] = None) -> Dict:
    """Module entry point (advanced_velocity_optimization.py:527-564)."""
    if radar_params is None:
        radar_params = {'fc': 77e9, 'lambda_c': 3e8 / 77e9, 'num_antennas': 8}
    optimizer = AdvancedVelocityOptimizer(**radar_params)
    results = optimizer.run_robust_optimization(target_associations, dt, previous_motion)
    logger.info(f"Advanced velocity optimization complete: {results['success']}")
    return results
