"""Solver options with the reference defaults.

Defaults follow ``adjust_defines.h:105-141`` (cminpack lmdif / lmder) and the
``-imageWidth`` flag default (cmd/arg_flags_solve_info.h, 2048 px).  Unlike
the reference command (``arg_flags_solve_info.cpp:99-230``) nothing here is
Maya-specific; the mapping flag -> field is 1:1.
"""
from __future__ import annotations

from . import abi

ITERATIONS_DEFAULT = 100
TAU_DEFAULT = 1.0
EPSILON_DEFAULT = 1e-6
DELTA_DEFAULT = 1e-4
IMAGE_WIDTH_DEFAULT = 2048.0


def make_options(solver_type=abi.SOLVER_TYPE_CMINPACK_LMDER, iterations=ITERATIONS_DEFAULT,
                 tau=TAU_DEFAULT, epsilon1=EPSILON_DEFAULT, epsilon2=EPSILON_DEFAULT,
                 epsilon3=EPSILON_DEFAULT, delta=DELTA_DEFAULT,
                 auto_diff_type=abi.AUTO_DIFF_TYPE_FORWARD, auto_param_scale=1,
                 scene_graph_mode=abi.SCENE_GRAPH_MODE_MAYA_DAG,
                 image_width=IMAGE_WIDTH_DEFAULT, accept_only_better=1, log_level=0,
                 robust_loss=0, robust_loss_type=abi.ROBUST_LOSS_TYPE_TRIVIAL,
                 robust_loss_scale=1.0, initial_error_avg=None):
    """Build an ``MmbaOptions`` (keyword names follow the mmSolver command flags).

    ``robust_loss`` is ``SolverOptions::solverSupportsRobustLoss`` (false for
    both cminpack types, adjust_defines.h:122,141); ``initial_error_avg`` (not None)
    hands over the initial error the caller measured
    (adjust_base.cpp:1080-1103)."""
    if tau < 0.0:  # arg_flags_solve_info.cpp:191-192 clamps tau to [0, 1]
        tau = 0.0
    if tau > 1.0:
        tau = 1.0
    if solver_type == abi.SOLVER_TYPE_CMINPACK_LMDIF:
        auto_diff_type = abi.AUTO_DIFF_TYPE_FORWARD  # lmdif only supports forward
    o = abi.MmbaOptions()
    o.solver_type = int(solver_type)
    o.iter_max = int(iterations)
    o.tau = float(tau)
    o.eps1 = float(epsilon1)
    o.eps2 = float(epsilon2)
    o.eps3 = float(epsilon3)
    o.delta = float(delta)
    o.auto_diff_type = int(auto_diff_type)
    o.auto_param_scale = int(auto_param_scale)
    o.scene_graph_mode = int(scene_graph_mode)
    o.image_width = float(image_width)
    o.accept_only_better = int(accept_only_better)
    o.log_level = int(log_level)
    o.robust_loss = int(robust_loss)
    o.robust_loss_type = int(robust_loss_type)
    o.robust_loss_scale = float(robust_loss_scale)
    o.initial_error_given = 0 if initial_error_avg is None else 1
    o.initial_error_avg = 0.0 if initial_error_avg is None else float(initial_error_avg)
    return o
