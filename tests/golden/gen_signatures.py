#!/usr/bin/env python3
"""Record the reference's public Python surface (module -> class -> method -> parameters/defaults)
as data, by parsing the reference sources with ``ast`` (nothing is imported or executed).
Output: tests/golden/ref_signatures.json (build container only)."""
import ast
import json
import os

REF = '/root/reference'
MODULES = {
    'src.radar_signal.dechirp': 'src/radar_signal/dechirp.py',
    'src.angle_estimation.angle_estimation': 'src/angle_estimation/angle_estimation.py',
    'src.velocity_solver.velocity_solver': 'src/velocity_solver/velocity_solver.py',
    'src.algorithms.robust_angle_estimation': 'src/algorithms/robust_angle_estimation.py',
    'src.robust_angle_estimation': 'src/robust_angle_estimation.py',
    'src.pose_integration.pose_integration': 'src/pose_integration/pose_integration.py',
    'src.algorithms.velocity_solver_improved': 'src/algorithms/velocity_solver_improved.py',
    'src.algorithms.advanced_velocity_optimization': 'src/algorithms/advanced_velocity_optimization.py',
    'evaluation.compute_pose_error': 'evaluation/compute_pose_error.py',
    'evaluation.compute_velocity_error': 'evaluation/compute_velocity_error.py',
}


def params(fn):
    a = fn.args
    names = [x.arg for x in a.args]
    defaults = [ast.unparse(d) for d in a.defaults]
    pad = [None] * (len(names) - len(defaults))
    return [[n, d] for n, d in zip(names, pad + defaults)]


def main():
    out = {}
    for mod, path in MODULES.items():
        tree = ast.parse(open(os.path.join(REF, path)).read())
        m = {}
        for node in tree.body:
            if isinstance(node, ast.ClassDef):
                m[node.name] = {f.name: params(f) for f in node.body if isinstance(f, ast.FunctionDef)}
            elif isinstance(node, ast.FunctionDef):
                m[node.name] = params(node)
        out[mod] = m
    json.dump(out, open(os.path.join(os.path.dirname(os.path.abspath(__file__)), 'ref_signatures.json'), 'w'),
              indent=1, sort_keys=True)


if __name__ == '__main__':
    main()
