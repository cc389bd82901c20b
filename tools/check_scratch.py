"""Fail when a hot kernel of the compiled planar arms uses scratch (private stack memory), in fp64 and in
fp32 (the precision modes of BASELINE configs 3 and 5).

Reads the output of `hipcc -Rpass-analysis=kernel-resource-usage` (stdin) and reports, per kernel,
VGPRs / scratch bytes per lane / occupancy.  A kernel whose name matches one of the hot families
below, compiled for a static model (Arm<n>) in fp64 or fp32, must have ScratchSize 0: the round-3
dynamics pruning once made the compiler move k_qp_grad's arrays to scratch (592 B per lane, 3x slower,
DESIGN.md 4d) without a single reported spill, and the fp32 instances kept rolled joint loops (their
arrays dynamically indexed, so in scratch) until the full-unroll threshold.
Usage: make -C trajoptmpcreference_amd/csrc check-scratch
"""
import re
import sys

# (k_ls_terms is not gated: it trades 348 B/lane of spill for a second wave per SIMD, measured faster,
# tmpc_fd.hip)
HOT = ("k_qp_grad", "k_qp_fd", "k_qp_minv", "k_ilqr_forward", "k_ilqr_backward", "k_qp<",
       "k_qpILi", "k_mpc_shift", "k_rollout")


def main():
    cur, res = None, {}
    for line in sys.stdin:
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            res[cur] = {}
            continue
        m = re.search(r"remark:\s+(VGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]): (\d+)", line)
        if m and cur:
            res[cur][m.group(1).split()[0]] = int(m.group(2))
    bad = []
    for k, v in sorted(res.items()):
        # fp64 / fp32 instances on a compiled model (...Arm6Ed... / ...Arm6Ef...), and the Riccati sweep
        # (...ILi6Ed... / ...ILi6Ef...)
        hot = any(h in k for h in HOT) and (re.search(r"Arm\d+E[df]", k) or re.search(r"k_ilqr_backwardILi\d+E[df]", k))
        # model-independent hot kernels: the soft-limit (G + rho I)^-1 of config 4 (its 2-link-only UrdfCost
        # branch once spilled the other instances) and the hard-limit PCG
        hot = hot or re.search(r"k_ginv_softILi\d+E|k_hard_pcgILi", k)
        if hot and v.get("ScratchSize", 0) > 0:
            bad.append((k, v))
        print(f"{k[:90]:90s} vgpr {v.get('VGPRs')} scratch {v.get('ScratchSize')} occ {v.get('Occupancy')}")
    for k, v in bad:
        print(f"SCRATCH in hot kernel: {k} {v}", file=sys.stderr)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
