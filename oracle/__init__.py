"""ORACLE — test infrastructure, not product code.

A CPU (NumPy) restatement of the reference's hot path
(VCA-EPFL/TrajoptMPCReference: RBDReference dynamics + gradients,
formKKTSystemBlocks / Schur complement, GBD-PCG, the SQP loop), each function
citing the reference file:line it follows.  It is pinned against golden
fixtures produced by running the reference itself in the build container
(tests/golden/make_golden.py -> tests/golden/*.npz).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import anything from this package, and only as the checker / the timed CPU
baseline.  The product package (trajoptmpcreference_amd) never imports it and
has no CPU fallback.
"""
