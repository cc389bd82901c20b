#!/usr/bin/env python3
"""Benchmark: MPC solves/s for arm6.urdf, N=64, SQP with PCG-SS (BASELINE.json).

One "step" = one batched SQP solve (TrajoptMPCReference.SQP semantics, run to
every problem's exit) of B independent problems of the §8d workload:
  arm6 (corrected), N=64, dt=0.1, Euler; QuadraticCost(I, 100 I,
  0.1 I, xg=0); problem i: q0 ~ U(-1,1)^6 from default_rng(seed0 + i),
  qd0 = 0, x = Euler rollout of u = 0; reference default options, fp64.
Inputs are resident in HBM before the timed region (each step restores the
initial trajectories with a device-to-device copy, inside the timed region).

Multi-GPU: `python bench.py --gpus N` starts the N ranks itself (one child
process per GPU with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT
set; the parent touches no GPU, prints rank 0's line and fails if any rank
fails); under a launcher that sets those variables (python -m
torch.distributed.run --nproc-per-node N bench.py --gpus N) each process is one
rank and WORLD_SIZE must equal --gpus.  Rank r solves global problems
[r B, (r+1) B) -- independent problems, no collective inside a solve, weak
scaling.  RCCL over xGMI through libtmpc's
tmpc_comm_* C ABI (trajoptmpcreference_amd/dist.py; no PyTorch) broadcasts the
initial states from rank 0, times the region with a barrier and the max over
ranks, and gathers every problem's exit code / iteration count to rank 0.

Checks carried in the line (rank 0): the CPU leg (oracle NumPy restatement,
`cpu_baseline`) solves the first S problems of the same workload and
`parity` compares them with the GPU's exit codes, SQP iteration counts and
per-QP PCG iteration counts; `kkt_residual` is SURVEY §8d's residual against
the reference's own first QP.
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0       # MI355X HBM3E (MI355X_MICROARCH.md: 8.0 TB/s)
FP64_PEAK_TFLOPS = 78.6     # MI355X fp64 vector (= fp64 matrix) peak
FP32_PEAK_TFLOPS = 157.3    # MI355X fp32 vector peak (non-packed FMA)
LDS_PEAK_GBS = 256 * 2.4 * 256   # 256 B/clk/CU (ds_read_b64/b128) x 2.4 GHz x 256 CUs
MALL_MEASURED_GBS = 8600.0  # Infinity-Cache-resident row gathers, chip-wide (MI355X_MICROARCH.md, Indexed rows)
CUS = 256


# Soft box-constraint presets (TrajoptConstraint.set_*_limits; |u| <= 0.5 and |q| <= 1.0 are
# active on part of the §8d workload: its unconstrained optima reach |u| ~ 1.5, |q| ~ 1).
LIMIT_PRESETS = {
    "none": {},
    "torque-al": {"torque": dict(mode="AUGMENTED_LAGRANGIAN", lb=-0.5, ub=0.5)},
    "torque-qp": {"torque": dict(mode="QUADRATIC_PENALTY", lb=-0.5, ub=0.5)},
    "torque-joint-al": {"torque": dict(mode="AUGMENTED_LAGRANGIAN", lb=-0.5, ub=0.5),
                        "joint": dict(mode="AUGMENTED_LAGRANGIAN", lb=-1.0, ub=1.0)},
    # hard limits (ACTIVE_SET rows in C, TrajoptMPCReference.py:238-248): the banded Schur path
    "torque-velocity-as": {"torque": dict(mode="ACTIVE_SET", lb=-0.5, ub=0.5),
                           "velocity": dict(mode="ACTIVE_SET", lb=-1.0, ub=1.0)},
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=4096, help="problems per GPU")
    ap.add_argument("--N", type=int, default=64)
    ap.add_argument("--links", type=int, default=6)
    ap.add_argument("--method", default="PCG-SS", help="SQP linear-system method: PCG-SS / PCG-BJ / PCG-J / S")
    ap.add_argument("--solver", default="sqp", choices=["sqp", "ilqr"],
                    help="sqp: the BASELINE metric; ilqr: BASELINE config 3 (same workload, iLQR)")
    ap.add_argument("--mpc-steps", type=int, default=0,
                    help="> 0: BASELINE config 5, one step = a receding-horizon loop of this many horizon solves "
                         "(use with --N 128 --solver ilqr --batch 8192)")
    ap.add_argument("--limits", default="none", choices=sorted(LIMIT_PRESETS),
                    help="soft box constraints: torque-al = BASELINE config 3 (with --solver ilqr), "
                         "torque-joint-al = config 4 (SQP-PCG with torque + joint limits)")
    ap.add_argument("--cost", default="quadratic", choices=["quadratic", "ee"],
                    help="ee: UrdfCost (SURVEY 8f row 4; 2-link only) with examples/twolinks.py's Q, QF, R, "
                         "xg = [-1, 1.5, 0, 0]; use with --links 2")
    ap.add_argument("--precision", default="fp64", choices=["fp64", "fp32", "mixed"],
                    help="tmpc_options.precision: fp32 = BASELINE config 3 (fp32 dynamics + Riccati), "
                         "mixed = config 5 (fp32 dynamics, fp64 PCG); the workload rollout stays fp64")
    ap.add_argument("--pcg-warm-start", action="store_true",
                    help="tmpc_options.pcg_warm_start: each PCG starts from the previous lambda (MPC loop)")
    ap.add_argument("--seed0", type=int, default=0)
    ap.add_argument("--q0-scale", type=float, default=1.0, help="start states q0 ~ U(-s, s)^n (SURVEY 8d: s = 1)")
    ap.add_argument("--erm", type=float, default=None,
                    help="options['expected_reduction_min_SQP_DDP'] (default 0.05; examples/twolinks.py uses -100)")
    ap.add_argument("--cpu-sample", type=int, default=-1, help="problems for the CPU baseline (-1: 40 per process, ~10-20 s)")
    ap.add_argument("--cpu-procs", type=int, default=0,
                    help="CPU-baseline processes (0: the cores this job may use -- the cgroup CPU quota when one "
                         "is set, else os.cpu_count())")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the config-4 line the default (headline) run adds after its own measurement")
    ap.add_argument("--secondary-steps", type=int, default=3)
    ap.add_argument("--secondary-parity", type=int, default=64, help="config-4 problems checked against the oracle")
    ap.add_argument("--no-hard-line", action="store_true",
                    help="skip the hard-limit line (ACTIVE_SET torque + velocity) after the headline")
    ap.add_argument("--hard-steps", type=int, default=3)
    ap.add_argument("--hard-parity", type=int, default=16, help="hard-limit problems checked against the oracle")
    return ap.parse_args(argv)


def initial_states(n, B, seed0, scale=1.0):
    q0 = np.zeros((B, n))
    for i in range(B):
        q0[i] = np.random.default_rng(seed0 + i).uniform(-scale, scale, n)
    return q0


def host_cores():
    """(cores this job may use, os.cpu_count(), basis): BASELINE.md section 3 asks for the host's cores;
    on a shared GPU box the job's share is its cgroup CPU quota (cpu.max), which os.cpu_count() -- the
    whole machine -- does not show."""
    total = os.cpu_count() or 1
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            share = max(1, int(int(quota) // int(period)))
            return min(share, total), total, "cgroup cpu.max quota"
    except (OSError, ValueError):
        pass
    try:
        aff = len(os.sched_getaffinity(0))
        return aff, total, "sched_getaffinity"
    except AttributeError:
        return total, total, "os.cpu_count()"


# ------------------------------------------------------------------ flop / byte models
def f_pcg_survey(N, nx):
    """f_pcg = 2*3*nx^2*N*2 + ~10*N*nx flop per PCG iteration (SpMV with the three
    S blocks of every block row and a three-block P^-1 apply, plus the vector work)."""
    return 2 * 3 * nx * nx * N * 2 + 10 * N * nx


def pcg_flops_impl(N, nx, method):
    """What k_qp executes per PCG iteration: SpMV over the 3N-2 stored S blocks; the
    preconditioner as implemented (SS: z = P_D (r - S_off P_D r), 4N-2 block products)."""
    spmv = 2 * (3 * N - 2) * nx * nx
    pre = {"PCG-J": N * nx, "PCG-BJ": 2 * N * nx * nx, "PCG-SS": 2 * (N + 2 * (N - 1) + N) * nx * nx,
           "PCG-0": 0}[method]
    return spmv + pre + 10 * N * nx


def b_pcg_survey(N, nx):
    """SURVEY §8(d) streaming model: b_pcg = 8 (2 (2N-1) nx^2 + 10 N nx) B per PCG iteration."""
    return 8 * (2 * (2 * N - 1) * nx * nx + 10 * N * nx)


def pcg_lds_bytes_per_iter(N, nx, method):
    """LDS bytes the array serves per PCG iteration (k_qp, one row per lane): SpMV reads 3 nx
    doubles per row; SS rebuilds its r block (2 nx) and reads w (2 nx) and t (nx); BJ 2 nx; plus
    the per-row vector stores (Ap, r, w, t, p for SS)."""
    reads = 3 * nx + {"PCG-J": 0, "PCG-0": 0, "PCG-BJ": 2 * nx, "PCG-SS": 5 * nx}[method]
    writes = {"PCG-J": 1, "PCG-0": 1, "PCG-BJ": 3, "PCG-SS": 5}[method]
    return 8 * N * nx * (reads + writes)


def qp_schur_flops(N, nx, nu):
    # per problem-QP: S blocks (A G A^T, B G B^T, A G), gamma, the diagonal-block inverses and dxu
    per_knot = 2 * (nx * nx * nx + nu * nu * nx + nx * nx * nx + nx * nu * nx + nx * nx * nx) + 2 * nx ** 3
    return N * per_knot


def workload_key(a):
    """file name of this workload's committed PMC summary, profiles/pmc/<key>.json"""
    key = f"{a.solver}_{a.method if a.solver == 'sqp' else 'ilqr'}_arm{a.links}_N{a.N}_B{a.batch}"
    if a.limits != "none":
        key += "_" + a.limits
    if a.mpc_steps > 0:
        key += f"_mpc{a.mpc_steps}"
    if a.precision != "fp64":
        key += "_" + a.precision
    if a.pcg_warm_start:
        key += "_warm"
    if a.cost != "quadratic":
        key += "_" + a.cost
    return key.replace("/", "-")


def measured_traffic(kernel_prefix, key, raw=False):
    """HBM bytes per launch of a kernel from THIS workload's rocprofv3 PMC summary (tools/pmc_summary.py
    writes profiles/pmc/<workload key>.json from separate FETCH_SIZE and WRITE_SIZE passes), or None.
    raw=True also returns the uncorrected FETCH_SIZE + WRITE_SIZE bytes."""
    path = os.path.join(ROOT, "profiles", "pmc", key + ".json")
    if not os.path.exists(path):
        return (None, None, None) if raw else (None, None)
    d = json.load(open(path))
    for k, v in d["kernels"].items():
        if k.startswith(kernel_prefix):
            src = d.get("source", os.path.relpath(path, ROOT))
            if raw:
                return v["hbm_bytes_per_launch"], src, (v["fetch_size_kib_raw"] + v["write_size_kib"]) * 1024
            return v["hbm_bytes_per_launch"], src
    return (None, None, None) if raw else (None, None)


# ------------------------------------------------------------------ CPU baseline (oracle = restatement)
def _cpu_solve(args):
    seed, n, N = args
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    from oracle import sqp as osqp
    from trajoptmpcreference_amd.urdf import parse_urdf, planar_arm_urdf
    m = parse_urdf(planar_arm_urdf(n))
    x, u = osqp.initial_problem(m, N, 0.1, seed)
    cost = osqp.QuadCost(np.eye(2 * n), 100 * np.eye(2 * n), 0.1 * np.eye(n), np.zeros(2 * n))
    r = osqp.sqp(m, cost, x, u, N, 0.1, "PCG-SS")
    return dict(exit_sqp=int(r["exit_sqp"]), sqp_iter=int(r["sqp_iter"]), pcg_iters=list(r["pcg_iters"]),
                x=r["x"], u=r["u"])


def cpu_baseline(n, N, sample, procs, seed0):
    ctx = mp.get_context("fork")
    jobs = [(seed0 + i, n, N) for i in range(sample)]
    t0 = time.perf_counter()
    with ctx.Pool(procs, initializer=os.environ.__setitem__, initargs=("OMP_NUM_THREADS", "1")) as pool:
        res = pool.map(_cpu_solve, jobs, chunksize=1)
    wall = time.perf_counter() - t0
    return sample / wall, wall, res


def _cpu_solve_config4(args):
    """the oracle's config-4 solve of one problem (tests/golden/make_oracle_fixtures.py job_config4)"""
    seed, n, N = args
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    from oracle import sqp as osqp
    from oracle.soft import SoftConstraints, SoftLimit
    from trajoptmpcreference_amd.urdf import parse_urdf, planar_arm_urdf
    m = parse_urdf(planar_arm_urdf(n))
    x, u = osqp.initial_problem(m, N, 0.1, seed)
    cost = osqp.QuadCost(np.eye(2 * n), 100 * np.eye(2 * n), 0.1 * np.eye(n), np.zeros(2 * n))
    lim = LIMIT_PRESETS["torque-joint-al"]
    lims = [SoftLimit(k, n, N, [v["lb"]] * n, [v["ub"]] * n, v["mode"]) for k, v in lim.items()]
    with np.errstate(all="ignore"):
        r = osqp.sqp(m, cost, x, u, N, 0.1, "PCG-SS", {}, SoftConstraints(lims))
    return dict(exit_sqp=int(r["exit_sqp"]), sqp_iter=int(r["sqp_iter"]), exit_soft=int(r["exit_soft"]),
                outer_iter=int(r["outer_iter"]), pcg_iters=list(r["pcg_iters"]), x=r["x"], u=r["u"])


def _cpu_solve_hard(args):
    """the oracle's solve of one problem under the hard preset torque-velocity-as, in the banded PCG's
    canonical summation order (oracle/hard.py pcg_canonical; tests/test_gpu_hard.py)"""
    seed, n, N = args
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    from oracle import hard as ohard
    from oracle import sqp as osqp
    from trajoptmpcreference_amd.urdf import parse_urdf, planar_arm_urdf
    m = parse_urdf(planar_arm_urdf(n))
    x, u = osqp.initial_problem(m, N, 0.1, seed)
    cost = osqp.QuadCost(np.eye(2 * n), 100 * np.eye(2 * n), 0.1 * np.eye(n), np.zeros(2 * n))
    lims = [ohard.HardLimit(k, n, v["lb"], v["ub"], v["mode"]) for k, v in LIMIT_PRESETS["torque-velocity-as"].items()]
    with np.errstate(all="ignore"):
        r = osqp.sqp(m, cost, x, u, N, 0.1, "PCG-SS", {}, hard=ohard.HardConstraints(lims), order="canonical")
    tr = r["trace"][1:]
    return dict(exit_sqp=int(r["exit_sqp"]), sqp_iter=int(r["sqp_iter"]), pcg_iters=list(r["pcg_iters"]),
                x=r["x"], u=r["u"], alpha=[float(t["alpha"]) for t in tr],
                succeeded=[bool(t["succeeded_line_search"]) for t in tr])


def _gpu_iterate(ctx, x0, u0, N, dt, method, gr, i, j):
    """the GPU's own iterate j of problem i (the same solve stopped after j iterations) and the rho its QP j
    used (the schedule of check_for_exit_or_error, TrajoptMPCReference.py:457-481, from the trace's
    line-search outcomes)"""
    o = ctx.options
    rho, drho = o.rho_init_SQP_DDP, 1.0
    for q in range(j):
        if gr["trace"]["succeeded_line_search"][i, q + 1]:
            drho = min(drho / o.rho_factor_SQP_DDP, 1.0 / o.rho_factor_SQP_DDP)
        else:
            drho = max(drho * o.rho_factor_SQP_DDP, o.rho_factor_SQP_DDP)
        rho = max(rho * drho, o.rho_min_SQP_DDP)
    xi, ui = x0[i:i + 1], u0[i:i + 1]
    if j > 0:
        keep = o.max_iter_SQP_DDP
        ctx.set_options(max_iter_SQP_DDP=j)
        try:
            rj = ctx.sqp_solve_batch(xi, ui, N, dt, method, with_trace=False)
        finally:
            ctx.set_options(max_iter_SQP_DDP=keep)
        xi, ui = rj["x"], rj["u"]
    return xi, ui, rho


def classify_hard_mismatch(ctx, x0, u0, N, dt, method, gr, i, ref):
    """Why a problem's hard-limit run differs from the oracle's, replayed on the GPU's own inputs
    (tests/test_gpu_hard.py does this for every QP):
      * "pcg_count": at the first QP j where the PCG counts differ, the GPU's own iterate j is re-solved on
        the device (tmpc_qp_batch) and the oracle's canonical-order PCG (oracle/hard.py pcg_canonical)
        runs on that QP's own S and gamma: it takes the GPU's count -- the runs' S differ in the last
        bits (the GPU's and the oracle's dynamics / Schur formation) on a count the summation order
        decides;
      * "line_search": every common QP's count agrees and the runs part at the first iteration j whose
        line-search outcome (alpha, success) differs: the oracle's line search (oracle/sqp.py
        line_search), run at the GPU's iterate j along the GPU's own direction for it, takes the GPU's
        outcome -- the runs' directions differ in the last bits (their QPs' S do), and the trial's
        acceptance is decided there;
      * None: not reproduced."""
    from oracle import hard as ohard
    from oracle import sqp as osqp
    from trajoptmpcreference_amd.urdf import parse_urdf, planar_arm_urdf
    ex, it = int(gr["exit_sqp"][i]), int(gr["sqp_iter"][i])
    g_counts = [int(v) for v in gr["trace"]["pcg_iters"][i, 1:it + (1 if ex == 3 else 0) + 1]]
    o_counts = list(ref["pcg_iters"])
    o = ctx.options
    nx = x0.shape[1]
    j = next((q for q in range(min(len(g_counts), len(o_counts))) if g_counts[q] != o_counts[q]), None)
    if j is not None:
        xi, ui, rho = _gpu_iterate(ctx, x0, u0, N, dt, method, gr, i, j)
        q = ctx.qp_batch(xi, ui, N, dt, np.array([rho]), method, want_blocks=False, xs=x0[i:i + 1, :, 0])
        if int(q["pcg_iters"][0]) != g_counts[j]:
            return None
        info = ctx.qp_hard_info(1, N)
        D, W = int(info["dim"][0]), int(info["W"])
        S = np.zeros((D, D))
        for off in range(2 * W + 1):
            a = np.arange(D)
            c = a - W + off
            ok = (c >= 0) & (c < D)
            S[a[ok], c[ok]] = info["S_band"][0][a[ok], off]
        _, it_c = ohard.pcg_canonical(S, info["gamma"][0, :D], nx, method[4:], o.exit_tolerance_linSys,
                                      o.max_iter_linSys)
        return "pcg_count" if it_c == g_counts[j] else None
    g_ls = [(float(gr["trace"]["alpha"][i, q + 1]), bool(gr["trace"]["succeeded_line_search"][i, q + 1]))
            for q in range(it)]
    o_ls = list(zip(ref["alpha"], ref["succeeded"]))
    j = next((q for q in range(min(len(g_ls), len(o_ls))) if g_ls[q] != o_ls[q]), None)
    if j is None:
        return None
    xi, ui, rho = _gpu_iterate(ctx, x0, u0, N, dt, method, gr, i, j)
    q = ctx.qp_batch(xi, ui, N, dt, np.array([rho]), method, want_blocks=False, xs=x0[i:i + 1, :, 0])
    n = nx // 2
    m = parse_urdf(planar_arm_urdf(n))
    cost = osqp.QuadCost(np.eye(nx), 100 * np.eye(nx), 0.1 * np.eye(n), np.zeros(nx))
    lims = [ohard.HardLimit(k, n, v["lb"], v["ub"], v["mode"]) for k, v in LIMIT_PRESETS["torque-velocity-as"].items()]
    hc = ohard.HardConstraints(lims)
    xs = x0[i, :, 0].copy()
    with np.errstate(all="ignore"):
        J = osqp.total_cost(cost, xi[0], ui[0], N, None)
        c = osqp.total_violation(m, xi[0], ui[0], xs, N, dt, hc)
        r1 = osqp.line_search(cost, m, xi[0], ui[0], xs, N, dt, q["dxul"][0], J, J + 10 * c, 10,
                              osqp.default_options({}), None, hc)
    return "line_search" if (float(r1["alpha"]), bool(r1["succeeded_line_search"])) == g_ls[j] else None


def parity_check(gpu, cpu):
    """GPU vs oracle on the same problems: exit code, SQP iterations and the per-QP PCG counts must be
    identical (integer parity); trajectories are compared relative to their magnitude."""
    mism, worst = [], 0.0
    for i, c in enumerate(cpu):
        ex, it = int(gpu["exit_sqp"][i]), int(gpu["sqp_iter"][i])
        nq = it + (1 if ex == 3 else 0)
        pcg = [int(v) for v in gpu["trace"]["pcg_iters"][i, 1:nq + 1]]
        if ex != c["exit_sqp"] or it != c["sqp_iter"] or pcg != c["pcg_iters"]:
            mism.append(i)
        for a, b in ((gpu["x"][i], c["x"]), (gpu["u"][i], c["u"])):
            worst = max(worst, float(np.max(np.abs(a - b))) / max(1.0, float(np.max(np.abs(b)))))
    return {"checked": len(cpu), "mismatches": len(mism), "mismatched_problems": mism[:16],
            "compared": "exit_sqp, sqp_iter, per-QP PCG iteration counts (exact); final x, u",
            "max_traj_rel_diff": worst}


# ------------------------------------------------------------------ KKT residual vs the reference (golden QP)
def kkt_residual_check(ctx, n):
    """|r_build - r_ref| for the first QP of arm6 N=64 seed 0, r = ||[G+rho I, C^T; C, 0] dxul - [g; c]||_inf
    computed identically on both sides; the reference's r comes from tests/golden."""
    path = os.path.join(ROOT, "tests", "golden", "qp_arm6fix_N64.npz")
    if n != 6 or not os.path.exists(path):
        return None
    d = np.load(path)
    N = d["x"].shape[1]
    nx, nu = 2 * n, n
    r = ctx.qp_batch(d["x"][None], d["u"][None], N, float(d["dt"]), float(d["rho"]), "PCG-SS", want_blocks=False)
    dxul = r["dxul"][0]
    nz = (nx + nu) * (N - 1) + nx
    G = np.zeros((nz, nz))
    for k in range(N - 1):
        G[k * (nx + nu):k * (nx + nu) + nx, k * (nx + nu):k * (nx + nu) + nx] = np.eye(nx)
        G[k * (nx + nu) + nx:(k + 1) * (nx + nu), k * (nx + nu) + nx:(k + 1) * (nx + nu)] = 0.1 * np.eye(nu)
    G[nz - nx:, nz - nx:] = 100 * np.eye(nx)
    G += float(d["rho"]) * np.eye(nz)
    C = np.zeros((nx * N, nz))
    C[:nx, :nx] = np.eye(nx)
    for k in range(N - 1):
        c0 = k * (nx + nu)
        C[(k + 1) * nx:(k + 2) * nx, c0:c0 + nx] = -d["A"][k]
        C[(k + 1) * nx:(k + 2) * nx, c0 + nx:c0 + nx + nu] = -d["B"][k]
        C[(k + 1) * nx:(k + 2) * nx, c0 + nx + nu:c0 + 2 * nx + nu] = np.eye(nx)
    K = np.block([[G, C.T], [C, np.zeros((nx * N, nx * N))]])
    rhs = np.concatenate([d["g"], d["c"]])
    r_build = float(np.max(np.abs(K @ dxul - rhs)))
    r_ref = float(d["kkt_res_SS"])
    return {"r_build": r_build, "r_ref": r_ref, "abs_diff": abs(r_build - r_ref),
            "pcg_iters_build": int(r["pcg_iters"][0]), "pcg_iters_ref": int(d["iters_SS"])}


def ilqr_backward_flops_per_knot(nx, nu):
    # V_xx [A B], A^T P, B^T [P R], Q_ux^T [K d] products + the per-lane Cholesky solves
    return 2 * (2 * nx ** 3 + 2 * nx * nx * nu + nu * nu * nx + nx * nx * nu) + 2 * (nx + 1) * nu * nu


def hard_limits(preset):
    """the preset has ACTIVE_SET / FULL_SET (hard) rows"""
    return any(v["mode"] in ("ACTIVE_SET", "FULL_SET") for v in LIMIT_PRESETS[preset].values())


def hard_roofline(a, kernels, hard_bytes):
    """Roofline of k_hard_pcg, the hard-limit path's dominant kernel.  `achieved` = the bytes the kernel
    itself counts (tmpc_kernel_bytes): everything it reads and writes beyond its registers and
    LDS -- per iteration the band entries not held in registers and the preconditioner blocks not held in
    LDS, gamma in, lambda out, the setup blocks -- / the average launch time, against the HBM peak.  After
    the first iteration those re-reads are L2 hits (a problem's streamed part is ~85 kB; 32 problems per
    XCD fit its 4 MB L2): `traffic`, the PMC bytes, is what reaches the fabric, and hbm_GBps / hbm_frac
    show how little HBM the kernel uses.  It is bound by one problem's iteration latency, not by memory."""
    hp = kernels["hard_pcg"]
    per_launch = hard_bytes / hp["launches"]
    avg_s = hp["avg_ms"] / 1e3
    ach = per_launch / avg_s / 1e9
    traffic, src = measured_traffic("void tmpc::k_hard_pcg<", workload_key(a))
    out = {"kernel": "k_hard_pcg", "bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": ach / HBM_PEAK_GBS, "traffic": traffic, "avg_launch_ms": hp["avg_ms"],
           "algorithmic_bytes_per_launch": per_launch,
           "bytes_basis": "counted by the kernel per problem: 8 B x (2 D + iterations x band entries not in "
                          "registers + (iterations + 1) x distinct preconditioner entries not in LDS + once: "
                          "register-held band entries, setup blocks), DESIGN.md 4f; served by L2 after the first "
                          "iteration",
           "note": "each row's first band entries stay in registers and the preconditioner blocks in LDS for "
                   "the whole solve, so memory is not what binds: one 16-wave workgroup per problem, the PCG "
                   "iteration's barrier-separated phases (DESIGN.md 4f)"}
    if traffic:
        out.update(hbm_GBps=traffic / avg_s / 1e9, hbm_frac=traffic / avg_s / 1e9 / HBM_PEAK_GBS,
                   traffic_source=src,
                   traffic_note="2 x FETCH_SIZE + WRITE_SIZE per launch; FETCH_SIZE includes Infinity-Cache hits")
    return out


def sqp_roofline(a, N, nx, nu, kernels, counters):
    """Roofline of the dominant kernel k_qp (Schur + PCG + dxu fused, one workgroup per problem).
    frac uses SURVEY §8(d)'s algorithmic flops (f_pcg per PCG iteration); the kernel keeps S and
    P^-1 in registers, so it is bound by fp64 VALU issue, LDS bandwidth and barrier latency, not
    by HBM: hbm_frac (PMC bytes) is reported beside it."""
    qp = kernels["qp"]
    per_launch_iters = int(counters[1]) / max(1, qp["launches"])
    per_launch_qps = int(counters[0]) / max(1, qp["launches"])
    avg_s = qp["avg_ms"] / 1000.0
    flops = per_launch_iters * f_pcg_survey(N, nx)
    ach = flops / avg_s / 1e12
    impl = per_launch_iters * pcg_flops_impl(N, nx, a.method) + per_launch_qps * qp_schur_flops(N, nx, nu)
    lds_bytes = per_launch_iters * pcg_lds_bytes_per_iter(N, nx, a.method)
    traffic, src = measured_traffic(f"void tmpc::k_qp<{nx // 2}, ", workload_key(a))
    if N * nx > 1024:
        traffic, src, raw = measured_traffic(f"void tmpc::k_qp<{nx // 2}, ", workload_key(a), raw=True)
        return gm_roofline(a, N, nx, qp, per_launch_iters, per_launch_qps, traffic, src, raw)
    out = {"kernel": "k_qp (Schur + PCG + dxu, fused)", "bound": "fp64-valu", "achieved": ach,
           "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": ach / FP64_PEAK_TFLOPS, "traffic": traffic,
           "avg_launch_ms": qp["avg_ms"], "pcg_iters_per_launch": per_launch_iters,
           "flops_basis": "SURVEY 8(d) f_pcg = 2*3*nx^2*N*2 + 10*N*nx flop per PCG iteration "
                          f"({f_pcg_survey(N, nx)} at N={N}, nx={nx}) x PCG iterations per launch",
           "algorithmic_flops_per_launch": flops,
           "impl_flops": {"per_launch": impl, "tflops": impl / avg_s / 1e12,
                          "frac": impl / avg_s / 1e12 / FP64_PEAK_TFLOPS,
                          "basis": "flops k_qp executes: SpMV over 3N-2 blocks, SS as 4N-2 block products, "
                                   "plus the Schur prologue / dxu epilogue"},
           "lds_model": {"achieved_GBps": lds_bytes / avg_s / 1e9, "peak_GBps": LDS_PEAK_GBS,
                         "frac": lds_bytes / avg_s / 1e9 / LDS_PEAK_GBS, "lds_bytes_per_launch": lds_bytes},
           "note": "bound label: the contract's enum has no fp64-VALU/LDS value; S and P^-1 stay in registers "
                   "so HBM is not the binding resource (hbm_frac)"}
    if traffic:
        gbs = traffic / avg_s / 1e9
        out.update(hbm_GBps=gbs, hbm_frac=gbs / HBM_PEAK_GBS, traffic_source=src)
    sb = per_launch_iters * b_pcg_survey(N, nx)
    out["streaming_model"] = {"bytes_per_launch": sb, "GBps": sb / avg_s / 1e9,
                              "note": "SURVEY 8(d) b_pcg: bytes a design streaming S and P^-1 from HBM every "
                                      "PCG iteration would move; this design never does"}
    return out


def gm_request_doubles_per_row(method):
    """doubles of S rows the GM kernel requests per row and PCG iteration (the P_kk^-1 row stays in
    registers): S p reads S_{k,k-1}, S_kk, S_{k,k+1} (3 nx); SS reads S_{k,k+/-1} again for
    t = r - S_off w: 5 nx; BJ / J / 0: 3 nx."""
    return {"PCG-SS": 5}.get(method, 3)


def gm_roofline(a, N, nx, qp, per_launch_iters, per_launch_qps, traffic, src, raw=None):
    """k_qp<..., GM> (N nx > 1024 rows, BASELINE config 5): the rows of S and P^-1 no longer fit a CU's
    registers and are re-read from HBM scratch (through L2 / MALL) every PCG iteration -- the design
    SURVEY 8(d)'s byte model prices, so the HBM roofline applies: achieved = b_pcg x PCG iterations per
    launch / launch time, against 8 TB/s; traffic = the PMC bytes of this workload (FETCH_SIZE doubled
    per the guide's gfx950 correction for 16-B/lane coalesced streams, which the rows are read as; the
    raw figure beside it).  FETCH_SIZE counts every L2 miss, Infinity-Cache (MALL) hits included, so it
    is an upper bound on HBM bytes; the kernel requests more than b_pcg (it re-reads S_off and P_kk
    inside an SS iteration: l2_request_model), and the difference is served by L2 / MALL."""
    avg_s = qp["avg_ms"] / 1000.0
    alg = per_launch_iters * b_pcg_survey(N, nx)
    ach = alg / avg_s / 1e9
    req = per_launch_iters * 8.0 * N * nx * nx * gm_request_doubles_per_row(a.method)
    # one problem per CU at a time (LDS); its rows of S in the scratch: [3 used of 4][nx / 2][rows][2] doubles
    resident = min(per_launch_qps, CUS) * 8.0 * 4 * nx * N * nx
    out = {"kernel": "k_qp<GM> (Schur + PCG + dxu, S / P^-1 rows in HBM scratch, re-read from L2 / Infinity Cache)",
           "bound": "hbm+mall", "achieved": ach,
           "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS, "traffic": traffic,
           "resident_set_MB": resident / 1e6,
           "mall_note": f"the rows of the problems in flight ({resident / 1e6:.0f} MB: at most one problem per CU) fit "
                        "the 256 MiB Infinity Cache, so after its prologue writes them a problem's PCG re-reads are "
                        "served on-die (L2 / MALL), not by HBM: achieved is an L2 + MALL rate, priced against the "
                        "HBM spec for comparability -- it is not HBM bandwidth (the guide measures 6.29 TB/s "
                        "achievable from HBM, 8.6 TB/s for Infinity-Cache-resident gathers)",
           "frac_of_mall_measured": ach / MALL_MEASURED_GBS,
           "avg_launch_ms": qp["avg_ms"], "pcg_iters_per_launch": per_launch_iters,
           "problem_qps_per_launch": per_launch_qps,
           "bytes_basis": f"SURVEY 8(d) b_pcg = 8 (2 (2N-1) nx^2 + 10 N nx) = {b_pcg_survey(N, nx)} B per PCG "
                          f"iteration at N={N}, nx={nx}, x PCG iterations per launch",
           "algorithmic_bytes_per_launch": alg,
           "l2_request_model": {"bytes_per_launch": req, "GBps": req / avg_s / 1e9,
                                "basis": f"{gm_request_doubles_per_row(a.method)} nx doubles of S / P^-1 rows "
                                         "requested per row and PCG iteration (bench.py gm_request_doubles_per_row)"}}
    if traffic:
        out.update(hbm_GBps=traffic / avg_s / 1e9, hbm_frac=traffic / avg_s / 1e9 / HBM_PEAK_GBS,
                   traffic_source=src,
                   traffic_note="2 x FETCH_SIZE + WRITE_SIZE; FETCH_SIZE counts L2 misses, Infinity-Cache (MALL) "
                                "hits included, so this bounds HBM bytes from above")
    if raw:
        out.update(traffic_raw=raw, traffic_raw_GBps=raw / avg_s / 1e9)
    return out


def _free_port_pair():
    """A free TCP port P with P + 1 free too (P: MASTER_PORT; P + 1: the RCCL id exchange, dist.py)."""
    import socket
    for _ in range(64):
        with socket.socket() as s0:
            s0.bind(("127.0.0.1", 0))
            p = s0.getsockname()[1]
            if p >= 65535:
                continue
            try:
                with socket.socket() as s1:
                    s1.bind(("127.0.0.1", p + 1))
                return p
            except OSError:
                continue
    raise RuntimeError("no free port pair for the rank rendezvous")


def launch_ranks(a, argv):
    """--gpus N > 1 with no launcher: one child process per GPU (rank r on GPU r), this process touching no
    GPU.  Rank 0's stdout (the JSON line) is forwarded; the exit status is non-zero if any rank fails (the
    others are then stopped)."""
    import subprocess
    import tempfile
    port = _free_port_pair()
    procs = []
    with tempfile.TemporaryFile(mode="w+") as out0:
        for r in range(a.gpus):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus),
                       LOCAL_WORLD_SIZE=str(a.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
            procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                          stdout=out0 if r == 0 else subprocess.DEVNULL))
        rcs = [None] * len(procs)
        while any(rc is None for rc in rcs):
            for r, p in enumerate(procs):
                if rcs[r] is None:
                    rcs[r] = p.poll()
            if any(rc not in (None, 0) for rc in rcs):   # a rank failed: stop the others, fail
                for r, p in enumerate(procs):
                    if rcs[r] is None:
                        p.kill()
                        rcs[r] = p.wait()
                        rcs[r] = rcs[r] if rcs[r] else -9
                break
            time.sleep(0.2)
        out0.seek(0)
        sys.stdout.write(out0.read())
        sys.stdout.flush()
    bad = [r for r, rc in enumerate(rcs) if rc != 0]
    if bad:
        print(f"bench.py: ranks {bad} failed (exit codes {[rcs[r] for r in bad]})", file=sys.stderr)
        return 1
    return 0


def _standin():
    """TMPC_BENCH_STANDIN=<path>: a test stand-in module (tests/bench_standin.py) supplying Context and
    make_comm, so the CPU test suite can run the multi-rank launch path without a GPU.  Never set by the
    driver's runs: unset, the bench runs libtmpc (and fails without a GPU)."""
    path = os.environ.get("TMPC_BENCH_STANDIN")
    if not path:
        return None
    import importlib.util
    spec = importlib.util.spec_from_file_location("tmpc_bench_standin", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(a, sys.argv[1:]))
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) != a.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={os.environ['WORLD_SIZE']} but --gpus {a.gpus}: pass the same N")
    from trajoptmpcreference_amd import _native, dist
    from trajoptmpcreference_amd.urdf import parse_urdf, planar_arm_urdf

    rank, world, local_rank = dist.env_ranks()
    n, N, B, dt = a.links, a.N, a.batch, 0.1
    nx, nu = 2 * n, n
    model = parse_urdf(planar_arm_urdf(n))
    standin = _standin()
    ctx = standin.Context(local_rank) if standin else _native.Context(local_rank)
    # every rank must run the same configuration: its hash rides on the RCCL id exchange (dist.py)
    cfg = dist.config_hash({k: v for k, v in sorted(vars(a).items()) if k != "cpu_procs"}, model.X0, model.Xa,
                           model.Xb, model.I, np.asarray(model.parent), bytes(ctx.options))
    comm = standin.make_comm(ctx, rank, world, cfg) if standin else dist.make_comm(ctx, rank, world, cfg)
    ctx.set_model(model)
    if a.cost == "ee":
        if n != 2:
            raise SystemExit("--cost ee needs --links 2 (UrdfCost is 2-link only, SURVEY F5)")
        ctx.set_cost_ee(np.eye(4), 100 * np.eye(4), 0.1 * np.eye(2), np.array([-1.0, 1.5, 0.0, 0.0]), None,
                        model.H0[:2], model.Ha[:2], model.Hb[:2])
    else:
        ctx.set_cost_quadratic(np.eye(nx), 100 * np.eye(nx), 0.1 * np.eye(nu), np.zeros(nx))
    limits = LIMIT_PRESETS[a.limits]
    ctx.set_box_limits(limits)

    # ---- workload: rank 0 draws every rank's start states, RCCL broadcast, own slice resident in HBM
    q0 = dist.scatter_from_root(comm, rank, B, lambda count: initial_states(n, count, a.seed0, a.q0_scale), (n,))
    x0 = np.zeros((B, nx, N))
    x0[:, :n, 0] = q0
    u0 = np.zeros((B, nu, N - 1))
    xb, ub = x0.nbytes, u0.nbytes
    d_x0, d_u0, d_x, d_u = ctx.alloc(xb), ctx.alloc(ub), ctx.alloc(xb), ctx.alloc(ub)
    ctx.h2d(d_x0, x0)
    ctx.h2d(d_u0, u0)
    ctx.rollout_device(B, N, dt, d_x0, d_u0)
    prec_id = {"fp64": 0, "fp32": 1, "mixed": 2}[a.precision]
    ctx.set_options(precision=prec_id, pcg_warm_start=int(a.pcg_warm_start))   # after the fp64 workload rollout
    if a.erm is not None:
        ctx.set_options(expected_reduction_min_SQP_DDP=float(a.erm))

    if a.mpc_steps > 0:
        K1 = a.mpc_steps
        d_xe, d_ue = ctx.alloc(B * nx * (K1 + 1) * 8), ctx.alloc(B * nu * K1 * 8)
        d_codes, d_iters = ctx.alloc(B * K1 * 4), ctx.alloc(B * K1 * 4)

    def solve(want_status=False):
        if a.mpc_steps > 0:
            ctx.mpc_batch_device(B, N, dt, "iLQR" if a.solver == "ilqr" else a.method, a.mpc_steps, d_x, d_u, d_xe,
                                 d_ue, d_codes, d_iters)
            if want_status:
                codes = np.zeros((B, a.mpc_steps), dtype=np.int32)
                its = np.zeros((B, a.mpc_steps), dtype=np.int32)
                ctx.d2h(codes, d_codes)
                ctx.d2h(its, d_iters)
                return codes.reshape(-1), its.reshape(-1)
            return None, None
        if a.solver == "ilqr":
            return ctx.ilqr_solve_batch_device(B, N, dt, d_x, d_u, want_status=want_status)
        return ctx.sqp_solve_batch_device(B, N, dt, d_x, d_u, a.method, want_status=want_status)

    def step():
        ctx.d2d(d_x, d_x0, xb)
        ctx.d2d(d_u, d_u0, ub)
        if limits:
            ctx.set_soft_state(B, N)   # every step starts from the initial mu / lambda / phi
        solve()

    for _ in range(a.warmup):
        step()
    ctx.synchronize()
    ctx.set_options(profile=1)
    ctx.reset_stats()
    counters = np.zeros(4, dtype=np.int64)
    comm.barrier()
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
        counters += np.array(ctx.solve_counters(), dtype=np.int64)
    ctx.synchronize()
    comm.barrier()
    t1 = time.perf_counter()
    elapsed = comm.max(t1 - t0)
    ctx.set_options(profile=0)
    hard_bytes = ctx.kernel_bytes("hard_pcg") if limits and a.method != "S" and hard_limits(a.limits) else None

    kernels = {}
    for name in ["qp_fd", "qp_minv", "qp_grad", "ginv", "qp", "schur", "btsolve", "dxu", "ls_terms", "ls_decide",
                 "hard_schur", "hard_pcg", "hard_direct", "ilqr_backward", "ilqr_forward", "ilqr_decide",
                 "mpc_shift"]:
        cnt, ms = ctx.kernel_stats(name)
        if cnt:
            kernels[name] = {"launches": cnt, "total_ms": ms, "avg_ms": ms / cnt}
    dominant = max(kernels, key=lambda k: kernels[k]["total_ms"])

    total_solves = B * a.steps * world * max(1, a.mpc_steps)
    value = total_solves / elapsed
    ms_per_step = 1000.0 * elapsed / a.steps

    # ---- status of one solve (exit codes / iteration counts), gathered from every rank over RCCL
    ctx.d2d(d_x, d_x0, xb)
    ctx.d2d(d_u, d_u0, ub)
    if limits:
        ctx.set_soft_state(B, N)
    exit_codes, iters = solve(want_status=True)
    g = dist.gather_summaries(comm, exit_codes=exit_codes.astype(np.int32), iters=iters.astype(np.int32))
    exit_all, iters_all = g["exit_codes"], g["iters"]

    # ---- PCIe-inclusive rate: the same batch through the host-array entry point (H2D + solve + D2H)
    pcie = None
    if a.solver == "sqp" and a.mpc_steps == 0 and not limits and a.cost == "quadratic":
        xh = np.empty((B, nx, N))
        ctx.d2h(xh, d_x0)
        ctx.synchronize()
        tp = time.perf_counter()
        ctx.sqp_solve_batch(xh, u0, N, dt, a.method, with_trace=False)
        tp = time.perf_counter() - tp
        pcie = {"value": B / tp, "unit": "solves/s", "ms_per_solve_batch": 1000.0 * tp,
                "note": "tmpc_sqp_solve_batch with host x/u (H2D, solve, D2H of x, u and the status arrays), "
                        "one batch, this GPU; `value` above is the HBM-resident rate"}
    comm.barrier()
    headline = a.solver == "sqp" and a.method == "PCG-SS" and a.mpc_steps == 0 and not limits and \
        a.cost == "quadratic" and N == 64 and a.precision == "fp64"
    # BASELINE config 4 beside the headline (after its measurement; every rank takes part)
    secondary = None
    if headline and not a.no_secondary and n == 6:
        secondary = run_secondary(a, ctx, comm, rank, world, n, N, B, dt, d_x0, d_u0, d_x, d_u, u0)
    hard_line = None
    if headline and not a.no_hard_line and n == 6:
        hard_line = run_hard_line(a, ctx, comm, rank, world, n, N, B, dt, d_x0, d_u0, d_x, d_u, u0)

    if rank != 0:
        comm.close()
        return

    name = 'iLQR' if a.solver == 'ilqr' else 'SQP ' + a.method
    if a.limits != "none":
        name += f", {'hard' if hard_limits(a.limits) else 'soft'} box constraints {a.limits}"
    if a.cost == "ee":
        name += ", UrdfCost end-effector cost (twolinks.py goal)"
    if a.mpc_steps > 0:
        name = f"receding-horizon MPC loop of {a.mpc_steps} horizon solves, {name}"
    if a.precision != "fp64":
        name += ", fp32 dynamics + Riccati" if a.precision == "fp32" else ", mixed fp32 dynamics / fp64 PCG"
    out = {
        "metric": ("MPC solves/sec (arm6.urdf, N=64, SQP-PCG) at 1/2/4/8 GPUs; KKT residual vs ref" if headline
                   else f"MPC solves/sec (arm{n}.urdf, N={N}, {name})"),
        "value": value, "unit": "solves/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": {"fp64": "f64", "fp32": "f32", "mixed": "f32 dynamics / f64 Schur-PCG"}[a.precision], "data": "synthetic (SURVEY §8d workload: seeded random start states, u=0 rollout)",
        "config": {"workload": f"arm{n}.urdf{' (joint6 fixed)' if n == 6 else ''} N={N} {a.solver.upper()} "
                               f"{'' if a.solver == 'ilqr' else a.method}, batch {B} per GPU"
                               + ("" if a.limits == "none" else f", limits {a.limits}")
                               + (", UrdfCost" if a.cost == "ee" else "")
                               + ("" if a.precision == "fp64" else f", precision {a.precision}")
                               + (f", MPC loop of {a.mpc_steps} steps" if a.mpc_steps > 0 else "")
                               + (", PCG warm start" if a.pcg_warm_start else ""),
                   "global_batch": B * world, "N": N, "method": a.method if a.solver == "sqp" else "iLQR",
                   "parallelism": f"shard{world} (RCCL broadcast of start states, gather of results)"},
    }
    roofline = None
    if a.solver == "sqp" and a.method.startswith("PCG") and a.mpc_steps == 0 and "qp" in kernels:
        roofline = sqp_roofline(a, N, nx, nu, kernels, counters)
    elif a.solver == "sqp" and a.method.startswith("PCG") and a.mpc_steps > 0 and "qp" in kernels and N * nx > 1024:
        # config 5 with SQP horizon solves: the GM QP kernel streams S / P^-1 rows (HBM roofline)
        roofline = sqp_roofline(a, N, nx, nu, kernels, counters)
    elif hard_bytes and "hard_pcg" in kernels:
        roofline = hard_roofline(a, kernels, hard_bytes)
    elif a.solver == "ilqr" and "ilqr_backward" in kernels:
        bw = kernels["ilqr_backward"]
        per_launch = int(counters[0]) / max(1, bw["launches"])
        flops = per_launch * (N - 1) * ilqr_backward_flops_per_knot(nx, nu)
        ach = flops / (bw["avg_ms"] / 1e3) / 1e12
        f32 = a.precision == "fp32"
        peak = FP32_PEAK_TFLOPS if f32 else FP64_PEAK_TFLOPS
        traffic, src = measured_traffic("void tmpc::k_ilqr_backward<", workload_key(a))
        roofline = {"kernel": "k_ilqr_backward", "bound": "fp32-valu" if f32 else "fp64-valu", "achieved": ach,
                    "peak": peak, "unit": "TFLOP/s", "frac": ach / peak, "traffic": traffic,
                    "algorithmic_flops_per_launch": flops, "avg_launch_ms": bw["avg_ms"],
                    "note": "sequential Riccati sweep, latency-bound (one 64-lane workgroup per problem)"}
        if traffic:
            roofline.update(hbm_GBps=traffic / (bw["avg_ms"] / 1e3) / 1e9, traffic_source=src)
        fw = kernels.get("ilqr_forward")
        if fw:
            ft, fsrc = measured_traffic("void tmpc::k_ilqr_forward<", workload_key(a))
            roofline["forward"] = {"kernel": "k_ilqr_forward", "avg_launch_ms": fw["avg_ms"], "traffic": ft,
                                   "hbm_GBps": ft / (fw["avg_ms"] / 1e3) / 1e9 if ft else None}
    out["roofline"] = roofline

    cpu, par = None, None
    if headline and not a.no_cpu_baseline and world == 1:
        share, total, basis = host_cores()
        procs = a.cpu_procs if a.cpu_procs > 0 else share
        sample = min(B, a.cpu_sample if a.cpu_sample > 0 else 40 * procs)
        v, wall, res = cpu_baseline(n, N, sample, procs, a.seed0)
        cpu = {"value": v, "unit": "solves/s", "cores": procs, "kind": "port",
               "sample": f"{sample} problems of the same workload (seeds {a.seed0}..{a.seed0 + sample - 1}), "
                         f"oracle NumPy restatement (no SymPy), {procs} processes x 1 BLAS thread, {wall:.1f} s",
               "cores_basis": f"{basis}: this job may use {share} cores of the {total} os.cpu_count() reports"}
        # the GPU's own results for those problems (rank 0's first `sample` problems), with trace
        gr = ctx.sqp_solve_batch(x0_host(ctx, d_x0, B, nx, N)[:sample], u0[:sample], N, dt, a.method)
        par = parity_check(gr, res)
    out["cpu_baseline"] = cpu
    if headline:
        out["parity"] = par
        out["kkt_residual"] = kkt_residual_check(ctx, n)
        out["pcie_inclusive"] = pcie
        out["value_basis"] = ("HBM-resident: inputs resident on the GPU before the timed region, each step a D2D "
                              "restore + one batched solve (the bench contract's definition); SURVEY 8(d) / "
                              "BASELINE.md section 3 count H2D/D2H in wall time -- that rate is pcie_inclusive")
        out["work"] = {"problem_qps_per_step": int(counters[0]) / a.steps,
                       "pcg_iters_per_step": int(counters[1]) / a.steps,
                       "grad_evals_per_step": int(counters[2]) / a.steps,
                       "ls_trials_per_qp": int(counters[3]) // max(1, a.steps)}
    out["kernels"] = kernels
    out["dominant_kernel"] = dominant
    # lock-step cost: every iteration launches the whole batch until its slowest problem exits
    it_name = "ilqr_decide" if a.solver == "ilqr" else "ls_decide"
    if it_name in kernels:
        out["lockstep"] = {"batch_iterations_per_solve": kernels[it_name]["launches"] / a.steps / max(1, a.mpc_steps),
                           "problem_iterations_mean": int(counters[0]) / (B * a.steps * max(1, a.mpc_steps))}
    out["exit_codes"] = {str(k): int(v) for k, v in zip(*np.unique(exit_all, return_counts=True))}
    out["iters_mean"] = float(np.mean(iters_all))
    out["iters_max"] = int(np.max(iters_all))
    out["problems_gathered"] = int(exit_all.size)
    if secondary is not None:
        out["secondary"] = secondary
    if hard_line is not None:
        out["hard_limits"] = hard_line
    print(json.dumps(out))
    comm.close()


def run_hard_line(a, ctx, comm, rank, world, n, N, B, dt, d_x0, d_u0, d_x, d_u, u0):
    """The headline workload under hard ACTIVE_SET torque + velocity limits (LIMIT_PRESETS
    "torque-velocity-as": constraint rows in C, the banded Schur path, TrajoptMPCReference.py:238-248),
    measured after the headline and the secondary, timed as the headline (barrier + synchronize around
    --hard-steps solves, max over ranks), with k_hard_pcg's roofline and the GPU's exit codes /
    iterations / per-QP PCG counts against the oracle (canonical order) on the first --hard-parity
    problems (rank 0)."""
    import copy
    nx, nu = 2 * n, n
    ah = copy.copy(a)
    ah.limits = "torque-velocity-as"
    ctx.set_box_limits(LIMIT_PRESETS[ah.limits])
    xb, ub = B * nx * N * 8, B * nu * (N - 1) * 8

    def step():
        ctx.d2d(d_x, d_x0, xb)
        ctx.d2d(d_u, d_u0, ub)
        ctx.sqp_solve_batch_device(B, N, dt, d_x, d_u, a.method)

    step()
    ctx.synchronize()
    ctx.set_options(profile=1)
    ctx.reset_stats()
    comm.barrier()
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.hard_steps):
        step()
    ctx.synchronize()
    comm.barrier()
    elapsed = comm.max(time.perf_counter() - t0)
    ctx.set_options(profile=0)
    hard_bytes = ctx.kernel_bytes("hard_pcg")
    kernels = {}
    for name in ["qp_fd", "qp_minv", "qp_grad", "ginv", "hard_schur", "hard_pcg", "dxu", "ls_terms", "ls_decide"]:
        cnt, ms = ctx.kernel_stats(name)
        if cnt:
            kernels[name] = {"launches": cnt, "total_ms": ms, "avg_ms": ms / cnt}
    ctx.d2d(d_x, d_x0, xb)
    ctx.d2d(d_u, d_u0, ub)
    exit_codes, iters = ctx.sqp_solve_batch_device(B, N, dt, d_x, d_u, a.method, want_status=True)
    from trajoptmpcreference_amd import dist
    dist.gather_summaries(comm, exit_codes=exit_codes.astype(np.int32), iters=iters.astype(np.int32))
    par = None
    if rank == 0 and a.hard_parity > 0:
        S = min(B, a.hard_parity)
        share, _, _ = host_cores()
        jobs = [(a.seed0 + i, n, N) for i in range(S)]
        with mp.get_context("fork").Pool(min(share, S), initializer=os.environ.__setitem__,
                                          initargs=("OMP_NUM_THREADS", "1")) as pool:
            res = pool.map(_cpu_solve_hard, jobs, chunksize=1)
        xh = x0_host(ctx, d_x0, B, nx, N)[:S]
        gr = ctx.sqp_solve_batch(xh, u0[:S], N, dt, a.method)
        par = parity_check(gr, res)
        why = {i: classify_hard_mismatch(ctx, xh, u0[:S], N, dt, a.method, gr, i, res[i])
               for i in par["mismatched_problems"]}
        par["replayed"] = {str(i): w for i, w in why.items()}
        par["unexplained"] = sum(1 for w in why.values() if w is None)
        par["note"] = ("oracle/sqp.py with oracle/hard.py's rows and pcg_canonical, the banded PCG's summation "
                       "order.  replayed: each mismatched problem replayed on the GPU's own inputs at the first "
                       "point the runs part (bench.classify_hard_mismatch): 'pcg_count' -- the canonical-order "
                       "PCG on the GPU's own S takes the GPU's count; 'line_search' -- the oracle's SQP "
                       "line search on the GPU's own iterate and direction takes the GPU's outcome")
    ctx.set_box_limits(None)
    value = B * a.hard_steps * world / elapsed
    return {"metric": f"MPC solves/sec (arm{n}.urdf, N={N}, SQP {a.method}, hard ACTIVE_SET torque + velocity "
                      "box limits)",
            "value": value, "unit": "solves/s", "n_gpus": world, "steps": a.hard_steps, "warmup": 1,
            "ms_per_step": 1000.0 * elapsed / a.hard_steps, "higher_is_better": True, "scaling": "weak",
            "config": {"workload": f"arm{n}.urdf (joint6 fixed) N={N} SQP {a.method}, batch {B} per GPU, limits "
                                   f"{ah.limits} (torque +-0.5, velocity +-1, ACTIVE_SET)",
                       "global_batch": B * world},
            "roofline": hard_roofline(ah, kernels, hard_bytes) if "hard_pcg" in kernels and hard_bytes else None,
            "kernels": kernels, "parity": par,
            "lockstep": {"batch_iterations_per_solve": kernels["ls_decide"]["launches"] / a.hard_steps}
            if "ls_decide" in kernels else None}


def run_secondary(a, ctx, comm, rank, world, n, N, B, dt, d_x0, d_u0, d_x, d_u, u0):
    """BASELINE config 4 beside the headline, measured after it (the headline's timed region is untouched):
    the same workload under soft torque + joint limits by augmented Lagrangian (LIMIT_PRESETS
    "torque-joint-al", SQP PCG-SS), timed exactly as the headline (barrier + synchronize around
    --secondary-steps solves, max over ranks), with its own kernel stats and k_qp roofline, and the GPU's
    exit codes / iterations / outer passes / per-QP PCG counts against the oracle on the first
    --secondary-parity problems (rank 0)."""
    import copy
    nx, nu = 2 * n, n
    a4 = copy.copy(a)
    a4.limits = "torque-joint-al"
    limits = LIMIT_PRESETS[a4.limits]
    ctx.set_box_limits(limits)
    xb, ub = B * nx * N * 8, B * nu * (N - 1) * 8

    def step():
        ctx.d2d(d_x, d_x0, xb)
        ctx.d2d(d_u, d_u0, ub)
        ctx.set_soft_state(B, N)
        ctx.sqp_solve_batch_device(B, N, dt, d_x, d_u, a.method)

    step()
    ctx.synchronize()
    ctx.set_options(profile=1)
    ctx.reset_stats()
    counters = np.zeros(4, dtype=np.int64)
    comm.barrier()
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.secondary_steps):
        step()
        counters += np.array(ctx.solve_counters(), dtype=np.int64)
    ctx.synchronize()
    comm.barrier()
    elapsed = comm.max(time.perf_counter() - t0)
    ctx.set_options(profile=0)
    kernels = {}
    for name in ["qp_fd", "qp_minv", "qp_grad", "ginv", "qp", "ls_terms", "ls_decide"]:
        cnt, ms = ctx.kernel_stats(name)
        if cnt:
            kernels[name] = {"launches": cnt, "total_ms": ms, "avg_ms": ms / cnt}
    ctx.d2d(d_x, d_x0, xb)
    ctx.d2d(d_u, d_u0, ub)
    ctx.set_soft_state(B, N)
    exit_codes, iters = ctx.sqp_solve_batch_device(B, N, dt, d_x, d_u, a.method, want_status=True)
    from trajoptmpcreference_amd import dist
    g = dist.gather_summaries(comm, exit_codes=exit_codes.astype(np.int32), iters=iters.astype(np.int32))
    par = None
    if rank == 0 and a.secondary_parity > 0:
        S = min(B, a.secondary_parity)
        share, _, _ = host_cores()
        jobs = [(a.seed0 + i, n, N) for i in range(S)]
        with mp.get_context("fork").Pool(min(share, S), initializer=os.environ.__setitem__,
                                          initargs=("OMP_NUM_THREADS", "1")) as pool:
            res = pool.map(_cpu_solve_config4, jobs, chunksize=1)
        ctx.set_soft_state(S, N)
        gr = ctx.sqp_solve_batch(x0_host(ctx, d_x0, B, nx, N)[:S], u0[:S], N, dt, a.method)
        par = parity_check(gr, res)
        soft_mism = [i for i, c in enumerate(res) if (int(gr["exit_soft"][i]), int(gr["outer_iter"][i]))
                     != (c["exit_soft"], c["outer_iter"])]
        par["mismatches"] += len([i for i in soft_mism if i not in par["mismatched_problems"]])
        par["compared"] += "; exit_soft, outer_iter (exact)"
    ctx.set_box_limits(None)
    value = B * a.secondary_steps * world / elapsed
    return {"metric": f"MPC solves/sec (arm{n}.urdf, N={N}, SQP {a.method}, soft torque + joint box limits by "
                      "augmented Lagrangian) -- BASELINE config 4's per-GPU slice",
            "value": value, "unit": "solves/s", "n_gpus": world, "steps": a.secondary_steps, "warmup": 1,
            "ms_per_step": 1000.0 * elapsed / a.secondary_steps, "higher_is_better": True, "scaling": "weak",
            "config": {"workload": f"arm{n}.urdf (joint6 fixed) N={N} SQP {a.method}, batch {B} per GPU, limits "
                                   f"{a4.limits} (torque +-0.5, joint +-1, AUGMENTED_LAGRANGIAN)",
                       "global_batch": B * world},
            "roofline": sqp_roofline(a4, N, nx, nu, kernels, counters) if "qp" in kernels else None,
            "kernels": kernels, "parity": par,
            "lockstep": {"batch_iterations_per_solve": kernels["ls_decide"]["launches"] / a.secondary_steps,
                         "problem_iterations_mean": int(counters[0]) / (B * a.secondary_steps)}
            if "ls_decide" in kernels else None,
            "exit_codes": {str(k): int(v) for k, v in zip(*np.unique(g["exit_codes"], return_counts=True))},
            "iters_mean": float(np.mean(g["iters"])), "iters_max": int(np.max(g["iters"]))}


def x0_host(ctx, d_x0, B, nx, N):
    x = np.empty((B, nx, N))
    ctx.d2h(x, d_x0)
    return x


if __name__ == "__main__":
    main()
