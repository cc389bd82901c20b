"""Config 3 fp32 / fp64 iLQR (8 problems of the oracle fixture) with the library TMPC_LIBRARY names:
prints exit codes and a digest of x, u so two builds can be compared bit for bit."""
import hashlib, sys, json
import numpy as np
sys.path.insert(0, "tests")
from conftest import arm_model, golden, quad_cost_arrays
from oracle import sqp as osqp
from trajoptmpcreference_amd import QuadraticCost, TrajoptConstraint, TrajoptMPCReference, URDFPlant, planar_arm_urdf

d = golden("oracle_config3_arm6_N64_ilqr_al.npz")
N = int(d["N"]); lb, ub = float(d["lb"]), float(d["ub"])
con = TrajoptConstraint(6, 6, 6, N)
con.set_torque_limits([ub] * 6, [lb] * 6, "AUGMENTED_LAGRANGIAN")
s = TrajoptMPCReference(URDFPlant(options={"path_to_urdf": planar_arm_urdf(6)}), QuadraticCost(*quad_cost_arrays(6)), con)
m = arm_model("arm6fix")
xs, us = zip(*[osqp.initial_problem(m, N, 0.1, int(q)) for q in d["seeds"]])
out = {}
for prec in ("fp64", "fp32"):
    opts = {"max_iter_softConstraints": int(d["max_iter_softConstraints"]),
            "max_iter_SQP_DDP": int(d["max_iter_SQP_DDP"]), "precision": prec}
    r = s.iLQR_batch(np.array(xs), np.array(us), N, 0.1, opts)
    out[prec] = dict(exit=[int(v) for v in r["exit_code"]], iters=[int(v) for v in r["iter"]],
                     outer=[int(v) for v in r["outer_iter"]],
                     xd=hashlib.sha256(np.ascontiguousarray(r["x"]).tobytes()).hexdigest()[:16],
                     ud=hashlib.sha256(np.ascontiguousarray(r["u"]).tobytes()).hexdigest()[:16])
print(json.dumps(out))
