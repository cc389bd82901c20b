"""MI355X-native batched SQP Schur-complement + GBD-PCG trajectory optimiser
with the plugin surface of VCA-EPFL/TrajoptMPCReference.

Host side: plain Python/NumPy classes that mirror the reference's
TrajoptPlant / TrajoptCost / TrajoptConstraint / PCG / TrajoptMPCReference
interfaces; compute: hand-written gfx950 HIP kernels in libtmpc.so behind a
ctypes C ABI (include/tmpc.h).  No CPU fallback.
"""
from .constraint import BoxConstraint, TrajoptConstraint
from .cost import QuadraticCost, TrajoptCost, UrdfCost
from .pcg import PCG
from .plant import PendulumPlant, TrajoptPlant, URDFPlant
from .solver import MPCSolverMethods, SQPSolverMethods, TrajoptMPCReference
from .urdf import RobotModel, parse_urdf, pendulum_urdf, planar_arm_urdf

__all__ = [
    "BoxConstraint", "TrajoptConstraint", "QuadraticCost", "TrajoptCost", "UrdfCost", "PCG", "TrajoptPlant", "URDFPlant",
    "PendulumPlant", "MPCSolverMethods", "SQPSolverMethods", "TrajoptMPCReference", "RobotModel", "parse_urdf",
    "pendulum_urdf", "planar_arm_urdf",
]
