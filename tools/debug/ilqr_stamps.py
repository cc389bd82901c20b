"""Per-phase cycle stamps of k_ilqr_backward (library built with -DTMPC_ILQR_STAMPS; run with
TMPC_LIBRARY=trajoptmpcreference_amd/libtmpc_istamps.so): one iLQR solve of B problems, the
device printf of block 0 per backward launch."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
import numpy as np
from conftest import arm_model, quad_cost_arrays
from trajoptmpcreference_amd import QuadraticCost, TrajoptMPCReference, URDFPlant, planar_arm_urdf
from oracle import sqp as osqp
B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
m = arm_model("arm6fix")
N = 64
xs, us = zip(*[osqp.initial_problem(m, N, 0.1, s) for s in range(B)])
s = TrajoptMPCReference(URDFPlant(options={"path_to_urdf": planar_arm_urdf(6)}), QuadraticCost(*quad_cost_arrays(6)))
r = s.iLQR_batch(np.array(xs), np.array(us), N, 0.1, {"max_iter_SQP_DDP": 3})
print("iters", r["iter"][:4], flush=True)
