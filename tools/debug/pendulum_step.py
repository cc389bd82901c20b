"""Debug: the GPU's third SQP step (QP 2) for the pendulum with ACTIVE_SET torque limits vs the oracle's."""
import sys
import numpy as np
sys.path.insert(0, ".")
from oracle import hard as ohard, sqp as osqp
from trajoptmpcreference_amd import PendulumPlant, QuadraticCost, TrajoptConstraint, TrajoptMPCReference

XG = np.array([3.14159, 0.0])
N = 20
np.set_printoptions(precision=6, linewidth=200)
for iters in (2, 3):
    plant = PendulumPlant()
    con = TrajoptConstraint(1, 1, 1, N)
    con.set_torque_limits([7.0], [-7.0], "ACTIVE_SET")
    solver = TrajoptMPCReference(plant, QuadraticCost(np.diag([1.0, 1.0]), np.diag([100.0, 100.0]), np.diag([0.1]), XG), con)
    x0, u0 = np.zeros((2, N)), np.zeros((1, N - 1))
    opts = {"expected_reduction_min_SQP_DDP": -100, "max_iter_SQP_DDP": iters + 1}
    res = solver.SQP(x0, u0, N, 0.1, "S", dict(opts))
    hard = ohard.HardConstraints([ohard.HardLimit("torque", 1, -7.0, 7.0, "ACTIVE_SET")])
    cost = osqp.QuadCost(np.diag([1.0, 1.0]), np.diag([100.0, 100.0]), np.diag([0.1]), XG)
    o = osqp.sqp(plant.model, cost, x0, u0, N, 0.1, "S", dict(opts), hard=hard)
    print("iters", iters + 1, "gpu", res[2], res[5], "oracle", o["exit_sqp"], o["sqp_iter"])
    print(" x gpu   ", res[0])
    print(" x oracle", o["x"])
    print(" u gpu   ", res[1])
    print(" u oracle", o["u"])
    print(" dxul oracle last", o["dxul"][-1][:3 * N])
