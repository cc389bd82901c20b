"""Debug: GPU vs oracle SQP trace for the pendulum with ACTIVE_SET torque limits."""
import sys
import numpy as np
sys.path.insert(0, ".")
from oracle import hard as ohard, sqp as osqp
from trajoptmpcreference_amd import PendulumPlant, QuadraticCost, TrajoptConstraint, TrajoptMPCReference

XG = np.array([3.14159, 0.0])
for method, lim in (("S", 7.0), ("S", 20.0), ("S", 1e9)):
    N = 20
    plant = PendulumPlant()
    con = TrajoptConstraint(1, 1, 1, N)
    con.set_torque_limits([lim], [-lim], "ACTIVE_SET")
    solver = TrajoptMPCReference(plant, QuadraticCost(np.diag([1.0, 1.0]), np.diag([100.0, 100.0]), np.diag([0.1]), XG), con)
    x0, u0 = np.zeros((2, N)), np.zeros((1, N - 1))
    opts = {"expected_reduction_min_SQP_DDP": -100}
    res = solver.SQP(x0, u0, N, 0.1, method, dict(opts))
    hard = ohard.HardConstraints([ohard.HardLimit("torque", 1, -lim, lim, "ACTIVE_SET")])
    cost = osqp.QuadCost(np.diag([1.0, 1.0]), np.diag([100.0, 100.0]), np.diag([0.1]), XG)
    o = osqp.sqp(plant.model, cost, x0, u0, N, 0.1, method, dict(opts), hard=hard)
    print(method, lim, "gpu", res[2], res[5], "oracle", o["exit_sqp"], o["sqp_iter"], "active", o["active_rows"])
    for i, (tg, to) in enumerate(zip(solver.trace, o["trace"])):
        print(f"  {i} alpha {tg['alpha']} / {to['alpha']}  J {tg['J']:.12g} / {to['J']:.12g}  c {tg['c']:.12g} / {to['c']:.12g}"
              f"  D {tg['D']} / {to['D']}")
