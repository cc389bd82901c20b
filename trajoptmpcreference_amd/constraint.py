"""TrajoptConstraint / BoxConstraint -- the reference's constraint plugin
surface (TrajoptConstraint.py:5-387).

This round the GPU solver runs the unconstrained path (the reference default
``TrajoptConstraint()``, the only configuration whose semantics are pinned:
SURVEY §0).  The classes keep the reference's constructor and setter
signatures so callers compose constraints the same way; solving with any
limit set raises NotImplementedError instead of silently ignoring it.
Box constraints with corrected vector semantics are the next row of the hot
path scope.
"""
from typing import List

import numpy as np

HARD_MODES = ("ACTIVE_SET", "FULL_SET")
SOFT_MODES = ("QUADRATIC_PENALTY", "AUGMENTED_LAGRANGIAN", "ADMM_PROJECTION")


class BoxConstraint:
    """lb <= x[:constraint_size] <= ub (TrajoptConstraint.py:5-51)."""

    def __init__(self, constraint_size: int = 0, num_timesteps: int = 0, upper_bounds: List[float] = (),
                 lower_bounds: List[float] = (), mode: str = "NONE", options=None):
        options = {} if options is None else options
        self.constraint_size = constraint_size
        self.num_timesteps = num_timesteps
        self.num_constraints = 2 * constraint_size * num_timesteps
        lblen, ublen = len(lower_bounds), len(upper_bounds)
        if (lblen != constraint_size and lblen != 1) or (ublen != constraint_size and ublen != 1):
            raise ValueError("please enter bounds of the size of constraint or constant 1")
        self.bounds = np.zeros(2 * constraint_size)
        self.bounds[:constraint_size] = lower_bounds
        self.bounds[constraint_size:] = upper_bounds
        if mode not in HARD_MODES + SOFT_MODES:
            raise ValueError("Invalid Constraint Mode. Options are [ACTIVE_SET, FULL_SET, QUADRATIC_PENALTY, "
                             "AUGMENTED_LAGRANGIAN, ADMM_PROJECTION]")
        self.mode = mode
        options.setdefault("quadratic_penalty_mu_init", 1e-2)
        options.setdefault("quadratic_penalty_mu_factor", 10.0)
        options.setdefault("quadratic_penalty_mu_max", 1e12)
        options.setdefault("augmentated_lagrangian_phi_init", 1e-2)
        options.setdefault("augmentated_lagrangian_phi_factor", 10.0)
        options.setdefault("jacobian_extra_columns_head", 0)
        options.setdefault("jacobian_extra_columns_tail", 0)
        self.options = options

    def is_hard_constraint_mode(self, mode=None):
        return (self.mode if mode is None else mode) in HARD_MODES

    def is_soft_constraint_mode(self, mode=None):
        return (self.mode if mode is None else mode) in SOFT_MODES


class TrajoptConstraint:
    """Joint / velocity / torque limits (TrajoptConstraint.py:178-387)."""

    def __init__(self, nq: int = 0, nv: int = 0, nu: int = 0, num_timesteps: int = 0):
        self.nq, self.nv, self.nu, self.num_timesteps = nq, nv, nu, num_timesteps
        self.joint_limits = None
        self.velocity_limits = None
        self.torque_limits = None

    def set_joint_limits(self, upper_bounds, lower_bounds, mode, options=None):
        options = {} if options is None else dict(options)
        options["jacobian_extra_columns_tail"] = self.nv + self.nu
        self.joint_limits = BoxConstraint(self.nq, self.num_timesteps - 1, upper_bounds, lower_bounds, mode, options)

    def set_velocity_limits(self, upper_bounds, lower_bounds, mode, options=None):
        options = {} if options is None else dict(options)
        options["jacobian_extra_columns_head"] = self.nq
        options["jacobian_extra_columns_tail"] = self.nu
        self.velocity_limits = BoxConstraint(self.nv, self.num_timesteps, upper_bounds, lower_bounds, mode, options)

    def set_torque_limits(self, upper_bounds, lower_bounds, mode, options=None):
        options = {} if options is None else dict(options)
        options["jacobian_extra_columns_head"] = self.nq + self.nv
        self.torque_limits = BoxConstraint(self.nu, self.num_timesteps - 1, upper_bounds, lower_bounds, mode, options)

    def has_any(self) -> bool:
        return any(c is not None for c in (self.joint_limits, self.velocity_limits, self.torque_limits))

    def total_soft_constraints(self, timestep=None):
        total = 0
        for c in (self.joint_limits, self.velocity_limits, self.torque_limits):
            if c is not None and c.is_soft_constraint_mode():
                total += c.num_constraints if timestep is None else c.constraint_size
        return total

    def total_hard_constraints(self, x=None, u=None, timestep=None):
        if any(c is not None and c.is_hard_constraint_mode()
               for c in (self.joint_limits, self.velocity_limits, self.torque_limits)):
            raise NotImplementedError("hard box constraints are not on the GPU path yet (SURVEY §8f row 1)")
        return 0

    def max_soft_constraint_value(self, x, u):
        if self.total_soft_constraints() > 0:
            raise NotImplementedError("soft box constraints are not on the GPU path yet (SURVEY §8f row 1)")
        return 0
