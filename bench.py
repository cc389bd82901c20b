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
                    help="skip the other BASELINE configurations' lines the default (headline) run adds after its "
                         "own measurement")
    ap.add_argument("--skip-lines", default="", help="comma-separated lines to skip: secondary, hard_limits, config2, "
                                                     "config3, config3_fp32, config5")
    ap.add_argument("--secondary-steps", type=int, default=16)
    ap.add_argument("--secondary-parity", type=int, default=64, help="config-4 problems checked against the oracle")
    ap.add_argument("--hard-steps", type=int, default=16)
    ap.add_argument("--hard-parity", type=int, default=64, help="hard-limit problems checked against the oracle")
    ap.add_argument("--config-steps", type=int, default=16, help="timed steps of the config 2 / 3 lines")
    ap.add_argument("--lockstep", action="store_true",
                    help="time each step as one lock-step batched solve (D2D restore + solve to every problem's "
                         "exit) instead of the continuous-batching stream")
    ap.add_argument("--substreams", type=int, default=1,
                    help="concurrent sub-streams of the headline's stream (tmpc_stream.substreams; the other lines use "
                         "their own tuned count, LINE_SUBSTREAMS)")
    ap.add_argument("--lockstep-steps", type=int, default=2,
                    help="lock-step steps timed beside each streamed line (its `lockstep` rate; 0: skip)")
    a = ap.parse_args(argv)
    a.skip_lines = [v for v in a.skip_lines.split(",") if v]
    return a


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
    if not getattr(a, "lockstep", True) and a.mpc_steps == 0:   # continuous batching: its own launches
        key += f"_stream{max(1, getattr(a, 'substreams', 1))}"
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


def classify_hard_mismatch(ctx, x0, u0, N, dt, method, gr, i, ref, limits="torque-velocity-as"):
    """Why a problem's hard-limit run differs from the oracle's, replayed at the first point the runs part,
    on the GPU's own inputs (tests/test_gpu_hard_arm6.py does this for every QP of every fixture problem).
    Returns a dict whose "kind" is:
      * "pcg_count": at the first QP j where the PCG counts differ, the GPU's own iterate j is re-solved on
        the device (tmpc_qp_batch) and takes the run's count, and the oracle's canonical-order PCG
        (oracle/hard.py pcg_canonical) on that QP's own S and gamma takes it too -- the runs' S differ in the
        last bits (the GPU's and the oracle's dynamics / Schur formation) on a count the rounding decides;
      * "line_search": every common QP's count agrees and the runs part at the first iteration j whose
        line-search outcome (alpha, success) differs.  At the GPU's iterate j the oracle's line search
        (oracle/sqp.py line_search) along the GPU's direction takes the GPU's outcome, AND along the
        oracle's own direction (its own dense KKT solve in the canonical PCG order at that iterate and rho)
        takes a different one: the two directions -- whose relative difference is reported -- decide the
        step, not the line search (whether that different outcome is exactly the oracle run's is reported);
      * None: not reproduced (the dict says which replay failed).
    The cost, limits and options are the bench's (the arguments), not fixed."""
    from oracle import hard as ohard
    from oracle import sqp as osqp
    from trajoptmpcreference_amd.urdf import parse_urdf, planar_arm_urdf
    ex, it = int(gr["exit_sqp"][i]), int(gr["sqp_iter"][i])
    g_counts = [int(v) for v in gr["trace"]["pcg_iters"][i, 1:it + (1 if ex == 3 else 0) + 1]]
    o_counts = list(ref["pcg_iters"])
    o = ctx.options
    nx = x0.shape[1]
    n = nx // 2
    j = next((q for q in range(min(len(g_counts), len(o_counts))) if g_counts[q] != o_counts[q]), None)
    if j is not None:
        xi, ui, rho = _gpu_iterate(ctx, x0, u0, N, dt, method, gr, i, j)
        q = ctx.qp_batch(xi, ui, N, dt, np.array([rho]), method, want_blocks=False, xs=x0[i:i + 1, :, 0])
        if int(q["pcg_iters"][0]) != g_counts[j]:
            return {"kind": None, "j": j, "failed": "the GPU's QP at its own iterate did not retake its count"}
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
        return {"kind": "pcg_count" if it_c == g_counts[j] else None, "j": j, "gpu_count": g_counts[j],
                "oracle_count": o_counts[j], "canonical_on_gpu_S": it_c}
    g_ls = [(float(gr["trace"]["alpha"][i, q + 1]), bool(gr["trace"]["succeeded_line_search"][i, q + 1]))
            for q in range(it + (1 if ex == 3 else 0))]
    o_ls = list(zip(ref["alpha"], ref["succeeded"]))
    j = next((q for q in range(min(len(g_ls), len(o_ls))) if g_ls[q] != o_ls[q]), None)
    if j is None:
        return {"kind": None, "failed": "no differing PCG count or line-search outcome"}
    xi, ui, rho = _gpu_iterate(ctx, x0, u0, N, dt, method, gr, i, j)
    q = ctx.qp_batch(xi, ui, N, dt, np.array([rho]), method, want_blocks=False, xs=x0[i:i + 1, :, 0])
    m = parse_urdf(planar_arm_urdf(n))
    cost = osqp.QuadCost(np.eye(nx), 100 * np.eye(nx), 0.1 * np.eye(n), np.zeros(nx))
    lims = [ohard.HardLimit(k, n, v["lb"], v["ub"], v["mode"]) for k, v in LIMIT_PRESETS[limits].items()]
    hc = ohard.HardConstraints(lims)
    xs = x0[i, :, 0].copy()
    opts = {k: getattr(o, k) for k in ("exit_tolerance_linSys", "max_iter_linSys", "alpha_factor_SQP_DDP",
                                       "alpha_min_SQP_DDP", "expected_reduction_min_SQP_DDP",
                                       "expected_reduction_max_SQP_DDP")}
    oo = osqp.default_options(opts)
    with np.errstate(all="ignore"):
        J = osqp.total_cost(cost, xi[0], ui[0], N, None)
        c = osqp.total_violation(m, xi[0], ui[0], xs, N, dt, hc)
        merit = J + o.merit_mu * c
        d_g = q["dxul"][0]
        r_g = osqp.line_search(cost, m, xi[0], ui[0], xs, N, dt, d_g, J, merit, o.merit_mu, oo, None, hc)
        G, g, Cm, cc = ohard.kkt_dense(m, cost, xi[0], ui[0], xs, N, dt, hc, None)
        d_o, _, _ = ohard.solve_qp_dense(G, g, Cm, cc, rho, method, oo, nx, {}, "canonical")
        r_o = osqp.line_search(cost, m, xi[0], ui[0], xs, N, dt, d_o, J, merit, o.merit_mu, oo, None, hc)
    npr = (nx + n) * (N - 1) + nx   # the primal part the line search steps along
    d_o = np.asarray(d_o, dtype=float).reshape(-1)[:npr]
    delta = float(np.max(np.abs(d_g[:npr] - d_o)) / max(1e-300, float(np.max(np.abs(d_o)))))
    out_g = (float(r_g["alpha"]), bool(r_g["succeeded_line_search"]))
    out_o = (float(r_o["alpha"]), bool(r_o["succeeded_line_search"]))
    gpu_ok = out_g == g_ls[j]
    ora_ok = out_o == o_ls[j]
    # explained: the oracle's line search reproduces the GPU's decision on the GPU's direction, and on the
    # oracle's own direction at the same iterate it decides differently -- the step is decided by the two
    # directions' difference (their QPs' S differ in the last bits; a capped PCG amplifies that), not by the
    # line search.  Whether the oracle's own direction then gives exactly the oracle RUN's outcome depends on
    # the oracle's iterate, which has the same rounding history, and on the host's BLAS (the dense KKT
    # formation's summation order): reported, not required.
    return {"kind": "line_search" if gpu_ok and out_o != g_ls[j] else None, "j": j, "gpu_outcome": g_ls[j],
            "oracle_direction_gives_oracle_run_outcome": ora_ok,
            "oracle_outcome": o_ls[j], "oracle_ls_on_gpu_direction": out_g, "oracle_ls_on_oracle_direction": out_o,
            "direction_rel_diff": delta, "pcg_counts_at_j": [g_counts[j] if j < len(g_counts) else None,
                                                            o_counts[j] if j < len(o_counts) else None]}


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
    return {"checked": len(cpu), "mismatches": len(mism), "mismatched_problems": mism[:64],
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


def hard_roofline(a, kernels, hard_bytes, counters=None):
    """Roofline of k_hard_pcg, the hard-limit path's dominant kernel: one 16-wave workgroup per problem keeps
    each row's first band entries in registers and the preconditioner blocks in LDS for the whole solve, so
    an iteration is bound by its LDS traffic and its two workgroup reductions' latency, not by
    HBM.  `achieved` = the LDS bytes an iteration serves (lds_model: per row and PCG iteration the 3 nx band
    entries' p, the SS preconditioner's 3 nx block entries and the 3 nx r entries they multiply, 9 nx doubles,
    plus 3 vector writes; D = N nx rows, the hard rows not counted, so a lower bound) x PCG iterations per launch
    / the HIP-event launch time, against the CUs' LDS bandwidth.  `traffic` / hbm_frac: the PMC bytes that reach
    HBM.  `self_counted`: the bytes the kernel reads and writes beyond registers and LDS
    (tmpc_kernel_bytes), served by L2 after the first iteration."""
    hp = kernels["hard_pcg"]
    avg_s = hp["avg_ms"] / 1e3
    nx, N = 2 * a.links, a.N
    iters = int(counters[1]) / max(1, hp["launches"]) if counters is not None else None
    lds = iters * 8.0 * N * nx * (9 * nx + 3) if iters is not None else None
    traffic, src = measured_traffic("void tmpc::k_hard_pcg<", workload_key(a))
    out = {"kernel": "k_hard_pcg", "bound": "lds",
           "bound_note": "LDS bandwidth and the two workgroup reductions' latency per PCG iteration (the contract's "
                         "enum has hbm / mfma only; HBM is what this kernel does NOT use: hbm_frac)",
           "achieved": lds / avg_s / 1e9 if lds else None, "peak": LDS_PEAK_GBS, "unit": "GB/s",
           "frac": lds / avg_s / 1e9 / LDS_PEAK_GBS if lds else None, "traffic": traffic,
           "avg_launch_ms": hp["avg_ms"], "pcg_iters_per_launch": iters, "lds_bytes_per_launch": lds,
           "lds_basis": "8 B x N nx rows x (9 nx + 3) per PCG iteration (DESIGN.md 4h: a row reads 3 nx p, 3 nx "
                        "preconditioner and 3 nx r entries from LDS)"}
    if hard_bytes:
        per_launch = hard_bytes / hp["launches"]
        out["self_counted"] = {"bytes_per_launch": per_launch, "GBps": per_launch / avg_s / 1e9,
                               "basis": "counted by the kernel per problem: 8 B x (2 D + iterations x band entries not "
                                        "in registers + (iterations + 1) x distinct preconditioner entries not in LDS "
                                        "+ once: register-held band entries, setup blocks), DESIGN.md 4f; L2 hits after "
                                        "the first iteration"}
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


def solver_name(a):
    """the stream / batch entry points' solver argument: "iLQR" or the SQP linear-system method"""
    return "iLQR" if a.solver == "ilqr" else a.method


def setup_workload(ctx, a):
    """model, cost, limits and options of workload `a` on the context (every line of the run re-does this)"""
    from trajoptmpcreference_amd.urdf import parse_urdf, planar_arm_urdf
    n = a.links
    nx, nu = 2 * n, n
    model = parse_urdf(planar_arm_urdf(n))
    ctx.set_model(model)
    if a.cost == "ee":
        if n != 2:
            raise SystemExit("--cost ee needs --links 2 (UrdfCost is 2-link only, SURVEY F5)")
        ctx.set_cost_ee(np.eye(4), 100 * np.eye(4), 0.1 * np.eye(2), np.array([-1.0, 1.5, 0.0, 0.0]), None,
                        model.H0[:2], model.Ha[:2], model.Hb[:2])
    else:
        ctx.set_cost_quadratic(np.eye(nx), 100 * np.eye(nx), 0.1 * np.eye(nu), np.zeros(nx))
    ctx.set_options(precision=0, pcg_warm_start=0)
    ctx.set_box_limits(LIMIT_PRESETS[a.limits])
    return model


def workload_inputs(ctx, comm, rank, a):
    """§8d workload of `a` for this rank: rank 0 draws every rank's start states, RCCL broadcast, the rank's
    slice resident in HBM, x = the fp64 Euler rollout of u = 0 on the device.  Returns the device buffers
    (initial x0, u0 and working x, u) and the host u0."""
    n, N, B, dt = a.links, a.N, a.batch, 0.1
    nx, nu = 2 * n, n
    from trajoptmpcreference_amd import dist
    q0 = dist.scatter_from_root(comm, rank, B, lambda count: initial_states(n, count, a.seed0, a.q0_scale), (n,))
    x0 = np.zeros((B, nx, N))
    x0[:, :n, 0] = q0
    u0 = np.zeros((B, nu, N - 1))
    d = dict(x0=ctx.alloc(x0.nbytes), u0=ctx.alloc(u0.nbytes), x=ctx.alloc(x0.nbytes), u=ctx.alloc(u0.nbytes),
             xb=x0.nbytes, ub=u0.nbytes)
    ctx.h2d(d["x0"], x0)
    ctx.h2d(d["u0"], u0)
    ctx.rollout_device(B, N, dt, d["x0"], d["u0"])
    # after the fp64 workload rollout: the line's precision and PCG warm start
    ctx.set_options(precision={"fp64": 0, "fp32": 1, "mixed": 2}[a.precision], pcg_warm_start=int(a.pcg_warm_start))
    if a.erm is not None:
        ctx.set_options(expected_reduction_min_SQP_DDP=float(a.erm))
    return d, u0


def free_inputs(ctx, d):
    for k in ("x0", "u0", "x", "u"):
        ctx.free(d[k])


def soft_limits(a):
    return a.limits != "none" and not hard_limits(a.limits)


def batch_solve(ctx, a, d, want_status=False, mpc=None):
    """one lock-step batched solve of the B resident problems from their initial trajectories (D2D restore
    first; soft limits from their initial constants); mpc: the MPC loop's output buffers"""
    B, N, dt = a.batch, a.N, 0.1
    ctx.d2d(d["x"], d["x0"], d["xb"])
    ctx.d2d(d["u"], d["u0"], d["ub"])
    if soft_limits(a):
        ctx.set_soft_state(B, N)
    if a.mpc_steps > 0:
        ctx.mpc_batch_device(B, N, dt, solver_name(a), a.mpc_steps, d["x"], d["u"], mpc["xe"], mpc["ue"],
                             mpc["codes"], mpc["iters"])
        if want_status:
            codes = np.zeros((B, a.mpc_steps), dtype=np.int32)
            its = np.zeros((B, a.mpc_steps), dtype=np.int32)
            ctx.d2h(codes, mpc["codes"])
            ctx.d2h(its, mpc["iters"])
            return codes.reshape(-1), its.reshape(-1)
        return None, None
    if a.solver == "ilqr":
        return ctx.ilqr_solve_batch_device(B, N, dt, d["x"], d["u"], want_status=want_status)
    return ctx.sqp_solve_batch_device(B, N, dt, d["x"], d["u"], a.method, want_status=want_status)


KERNEL_NAMES = ["qp_fd", "qp_minv", "qp_grad", "ginv", "qp", "schur", "btsolve", "dxu", "ls_terms", "ls_decide",
                "hard_schur", "hard_pcg", "hard_direct", "ilqr_backward", "ilqr_forward", "ilqr_decide", "mpc_shift",
                "soft_outer", "init_merit"]


def kernel_table(ctx):
    kernels = {}
    for name in KERNEL_NAMES:
        cnt, ms = ctx.kernel_stats(name)
        if cnt:
            kernels[name] = {"launches": cnt, "total_ms": ms, "avg_ms": ms / cnt}
    return kernels


def measure(ctx, comm, a, d, steps, warmup, stream, sbuf=None, mpc=None, substreams=1):
    """The timed region of one line: `warmup` untimed steps, then `steps` timed ones between barrier +
    synchronize, the max over ranks.  stream: the steps' B x steps problems go through the B slots of one
    continuous-batching solve (tmpc_*_solve_stream_device: problem p starts from resident input p % B,
    results to the sbuf output rows); else each step is a D2D restore + one lock-step batched solve.
    Returns (elapsed s, work counters, kernel table, k_hard_pcg's counted bytes or None)."""
    B, N, dt = a.batch, a.N, 0.1

    def stream_solve(copies):
        ctx.solve_stream_device(solver_name(a), B * copies, B, N, dt, d["x0"], d["u0"], B, sbuf["x"], sbuf["u"],
                                sbuf["st"], substreams=substreams)

    if stream:
        if warmup > 0:
            stream_solve(warmup)
    else:
        for _ in range(warmup):
            batch_solve(ctx, a, d, mpc=mpc)
    ctx.synchronize()
    ctx.set_options(profile=1)
    ctx.reset_stats()
    counters = np.zeros(4, dtype=np.int64)
    comm.barrier()
    ctx.synchronize()
    t0 = time.perf_counter()
    if stream:
        stream_solve(steps)
        counters += np.array(ctx.solve_counters(), dtype=np.int64)
    else:
        for _ in range(steps):
            batch_solve(ctx, a, d, mpc=mpc)
            counters += np.array(ctx.solve_counters(), dtype=np.int64)
    ctx.synchronize()
    comm.barrier()
    elapsed = comm.max(time.perf_counter() - t0)
    ctx.set_options(profile=0)
    if not stream:
        counters[3] = counters[3] // max(1, steps)   # line-search trials per QP (each solve reports it)
    hard_bytes = ctx.kernel_bytes("hard_pcg") if hard_limits(a.limits) and a.method != "S" else None
    return elapsed, counters, kernel_table(ctx), hard_bytes


def stream_buffers(ctx, a, copies):
    n, N, B = a.links, a.N, a.batch
    P = B * copies
    return dict(x=ctx.alloc(P * 2 * n * N * 8), u=ctx.alloc(P * n * (N - 1) * 8), st=ctx.alloc(P * 4 * 4), P=P)


def free_stream_buffers(ctx, sbuf):
    for k in ("x", "u", "st"):
        ctx.free(sbuf[k])


def stream_check(ctx, a, d, sbuf, copies, ex_b, it_b, xb):
    """The streamed problems against the lock-step batch solve of the same inputs (ex_b, it_b, xb: its exit
    codes, iteration counts and x): every stream problem's exit code and iteration count, and the final x of
    the first and the last copy of the batch bitwise (each problem's operations are the batch solve's)."""
    n, N, B = a.links, a.N, a.batch
    P = B * copies
    st = np.empty((P, 4), dtype=np.int32)
    ctx.d2h(st, sbuf["st"])
    mism = int(np.sum((st[:, 0] != np.tile(ex_b, copies)) | (st[:, 1] != np.tile(it_b, copies))))
    xs = np.empty((B, 2 * n, N))
    xm = []
    for c in sorted({0, copies - 1}):
        ctx.d2h(xs, sbuf["x"], offset=c * xs.nbytes)
        xm.append(int(np.sum(np.any(xs != xb, axis=(1, 2)))))
    return {"problems": P, "status_mismatches": mism, "x_copies_compared": sorted({0, copies - 1}),
            "x_mismatches": int(sum(xm)),
            "compared": "each streamed problem's exit code and iteration count against the lock-step batch solve of "
                        "its input; final x of the first and last copies bitwise"}


STREAM_BASIS = ("continuous batching (tmpc_sqp_solve_stream_device / tmpc_ilqr_solve_stream_device): the timed "
                "region solves steps x B problems (problem p starts from resident input p mod B) through B resident "
                "slots; a slot whose problem exits takes the next pending one in the same batch iteration, so the "
                "GPU never runs a near-empty lock-step tail.  Inputs resident in HBM before the timed region; every "
                "problem's results (x, u, exit code, iterations) are written to its own output rows.  ms_per_step = "
                "time / steps, i.e. per B problems.  Each problem's results equal its lock-step batch solve's "
                "bitwise (stream_check; tests/test_gpu_stream.py).  lockstep: the same workload one batch at a "
                "time (D2D restore + solve to every problem's exit), the round-5 definition")


def run_line(ctx, comm, rank, world, a, steps, warmup, stream, lockstep_steps, substreams=1):
    """Measure workload `a` (B = a.batch problems per rank): the line's value (solves/s over all ranks), its
    kernel table and work counters, the stream's check against the lock-step solve, and the lock-step rate.
    Returns (line dict, device inputs, host u0, the lock-step batch's status / x)."""
    setup_workload(ctx, a)
    d, u0 = workload_inputs(ctx, comm, rank, a)
    B, N = a.batch, a.N
    mpc = None
    if a.mpc_steps > 0:
        n = a.links
        K1 = a.mpc_steps
        mpc = dict(xe=ctx.alloc(B * 2 * n * (K1 + 1) * 8), ue=ctx.alloc(B * n * K1 * 8),
                   codes=ctx.alloc(B * K1 * 4), iters=ctx.alloc(B * K1 * 4))
        stream = False   # the MPC loop's horizon solves are lock-step batches (tmpc_mpc_batch_device)
    sbuf = stream_buffers(ctx, a, max(steps, warmup, 1)) if stream else None
    elapsed, counters, kernels, hard_bytes = measure(ctx, comm, a, d, steps, warmup, stream, sbuf, mpc, substreams)
    units = max(1, a.mpc_steps)
    value = B * steps * world * units / elapsed
    line = {"value": value, "unit": "solves/s", "n_gpus": world, "steps": steps, "warmup": warmup,
            "ms_per_step": 1000.0 * elapsed / steps, "higher_is_better": True, "scaling": "weak",
            "mode": "stream" if stream else ("lockstep MPC loop" if mpc else "lockstep")}
    if stream:
        line["substreams"] = substreams
    # the lock-step batch solve of the same inputs: status for the gather and the stream check
    ex_b, it_b = batch_solve(ctx, a, d, want_status=True, mpc=mpc)
    if stream:
        xb = np.empty((B, 2 * a.links, N))
        ctx.d2h(xb, d["x"])
        line["stream_check"] = stream_check(ctx, a, d, sbuf, steps, ex_b, it_b, xb)   # the timed stream's rows
        free_stream_buffers(ctx, sbuf)
        if lockstep_steps > 0:
            el, _, _, _ = measure(ctx, comm, a, d, lockstep_steps, 1, False)
            line["lockstep"] = {"value": B * lockstep_steps * world / el, "ms_per_step": 1000.0 * el / lockstep_steps,
                                "steps": lockstep_steps}
    it_name = "ilqr_decide" if a.solver == "ilqr" else "ls_decide"
    if it_name in kernels:
        line["batch_iterations"] = {
            "per_step": kernels[it_name]["launches"] / steps / units,
            "problem_iterations_mean": int(counters[0]) / (B * steps * units),
            "slot_utilization": int(counters[0]) / max(1, kernels[it_name]["launches"] * B)}
    line["work"] = {"problem_qps_per_step": int(counters[0]) / steps, "pcg_iters_per_step": int(counters[1]) / steps,
                    "grad_evals_per_step": int(counters[2]) / steps, "ls_trials_per_qp": int(counters[3])}
    line["kernels"] = kernels
    line["dominant_kernel"] = max(kernels, key=lambda k: kernels[k]["total_ms"]) if kernels else None
    from trajoptmpcreference_amd import dist
    g = dist.gather_summaries(comm, exit_codes=ex_b.astype(np.int32), iters=it_b.astype(np.int32))
    line["exit_codes"] = {str(k): int(v) for k, v in zip(*np.unique(g["exit_codes"], return_counts=True))}
    line["iters_mean"] = float(np.mean(g["iters"]))
    line["iters_max"] = int(np.max(g["iters"]))
    line["problems_gathered"] = int(g["exit_codes"].size)
    if mpc:
        for k in ("xe", "ue", "codes", "iters"):
            ctx.free(mpc[k])
    return line, d, u0, counters, kernels, hard_bytes


def line_roofline(a, N, nx, nu, kernels, counters, hard_bytes=None):
    if a.solver == "sqp" and a.method.startswith("PCG") and "qp" in kernels and (a.mpc_steps == 0 or N * nx > 1024):
        return sqp_roofline(a, N, nx, nu, kernels, counters)
    if hard_limits(a.limits) and "hard_pcg" in kernels:
        return hard_roofline(a, kernels, hard_bytes, counters)
    if a.solver == "ilqr" and "ilqr_backward" in kernels:
        bw = kernels["ilqr_backward"]
        per_launch = int(counters[0]) / max(1, bw["launches"])
        flops = per_launch * (N - 1) * ilqr_backward_flops_per_knot(nx, nu)
        ach = flops / (bw["avg_ms"] / 1e3) / 1e12
        f32 = a.precision == "fp32"
        peak = FP32_PEAK_TFLOPS if f32 else FP64_PEAK_TFLOPS
        traffic, src = measured_traffic("void tmpc::k_ilqr_backward<", workload_key(a))
        r = {"kernel": "k_ilqr_backward", "bound": "fp32-valu" if f32 else "fp64-valu", "achieved": ach,
             "peak": peak, "unit": "TFLOP/s", "frac": ach / peak, "traffic": traffic,
             "algorithmic_flops_per_launch": flops, "avg_launch_ms": bw["avg_ms"],
             "note": "sequential Riccati sweep, latency-bound (one 64-lane wave per problem)" + (
                 "; fp32 state and Cholesky, the Q products on the fp64 matrix cores from fp32 operands "
                 "(k_ilqr_backward<NJ, float, true>), priced against the fp32 VALU peak" if f32 else
                 "; Q products on v_mfma_f64_16x16x4f64")}
        if traffic:
            r.update(hbm_GBps=traffic / (bw["avg_ms"] / 1e3) / 1e9, traffic_source=src)
        fw = kernels.get("ilqr_forward")
        if fw:
            ft, fsrc = measured_traffic("void tmpc::k_ilqr_forward<", workload_key(a))
            r["forward"] = {"kernel": "k_ilqr_forward", "avg_launch_ms": fw["avg_ms"], "traffic": ft,
                            "hbm_GBps": ft / (fw["avg_ms"] / 1e3) / 1e9 if ft else None}
        return r
    return None


def line_config(a, world, name):
    B = a.batch
    return {"workload": f"arm{a.links}.urdf{' (joint6 fixed)' if a.links == 6 else ''} N={a.N} {name}, batch {B} per GPU"
                        + ("" if a.limits == "none" else f", limits {a.limits}")
                        + (", UrdfCost" if a.cost == "ee" else "")
                        + ("" if a.precision == "fp64" else f", precision {a.precision}")
                        + (f", MPC loop of {a.mpc_steps} steps" if a.mpc_steps > 0 else "")
                        + (", PCG warm start" if a.pcg_warm_start else ""),
            "global_batch": B * world, "N": a.N, "method": a.method if a.solver == "sqp" else "iLQR",
            "parallelism": f"shard{world} (RCCL broadcast of start states, gather of results)"}


def workload_name(a):
    name = 'iLQR' if a.solver == 'ilqr' else 'SQP ' + a.method
    if a.limits != "none":
        name += f", {'hard' if hard_limits(a.limits) else 'soft'} box constraints {a.limits}"
    if a.cost == "ee":
        name += ", UrdfCost end-effector cost (twolinks.py goal)"
    if a.mpc_steps > 0:
        name = f"receding-horizon MPC loop of {a.mpc_steps} horizon solves, {name}"
    if a.precision != "fp64":
        name += ", fp32 dynamics + Riccati" if a.precision == "fp32" else ", mixed fp32 dynamics / fp64 PCG"
    return name


def is_headline(a):
    return a.solver == "sqp" and a.method == "PCG-SS" and a.mpc_steps == 0 and a.limits == "none" and \
        a.cost == "quadratic" and a.N == 64 and a.precision == "fp64" and a.links == 6


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
    stream = not a.lockstep and a.mpc_steps == 0
    line, d, u0, counters, kernels, hard_bytes = run_line(ctx, comm, rank, world, a, a.steps, a.warmup, stream,
                                                          a.lockstep_steps if stream else 0, a.substreams)
    headline = is_headline(a)
    # ---- PCIe-inclusive rate: the same steps x B problems with host inputs and outputs (H2D of x0 / u0, the
    # stream, D2H of every problem's x, u and status) -- BASELINE.md section 3's wall-time definition
    pcie = None
    if headline:
        xh = x0_host(ctx, d["x0"], B, nx, N)
        pcie = pcie_inclusive(ctx, a, xh, u0, stream)
    comm.barrier()
    extra = {}
    if headline and not a.no_secondary:
        extra = run_config_lines(ctx, comm, rank, world, a)
    if rank != 0:
        comm.close()
        return
    out = {
        "metric": ("MPC solves/sec (arm6.urdf, N=64, SQP-PCG) at 1/2/4/8 GPUs; KKT residual vs ref" if headline
                   else f"MPC solves/sec (arm{n}.urdf, N={N}, {workload_name(a)})"),
        "value": line["value"], "unit": "solves/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": line["ms_per_step"], "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": {"fp64": "f64", "fp32": "f32", "mixed": "f32 dynamics / f64 Schur-PCG"}[a.precision],
        "data": "synthetic (SURVEY §8d workload: seeded random start states, u=0 rollout)",
        "config": line_config(a, world, f"{a.solver.upper()} {'' if a.solver == 'ilqr' else a.method}"),
    }
    if standin:
        out["standin"] = os.environ.get("TMPC_BENCH_STANDIN")   # a test stand-in context, not libtmpc
    out["roofline"] = line_roofline(a, N, nx, nu, kernels, counters, hard_bytes)
    if headline:
        out["value_pcie_inclusive"] = pcie["value"] if pcie else None
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
        gr = ctx.sqp_solve_batch(x0_host(ctx, d["x0"], B, nx, N)[:sample], u0[:sample], N, dt, a.method)
        par = parity_check(gr, res)
    out["cpu_baseline"] = cpu
    if headline:
        out["parity"] = par
        out["kkt_residual"] = kkt_residual_check(ctx, n)
        out["pcie_inclusive"] = pcie
    out["value_basis"] = STREAM_BASIS if stream else (
        "lock-step: each step a D2D restore + one batched solve to every problem's exit" +
        (" (MPC loop: a step = the receding-horizon loop over the batch)" if a.mpc_steps else ""))
    for k in ("mode", "stream_check", "lockstep", "batch_iterations", "work", "kernels", "dominant_kernel",
              "exit_codes", "iters_mean", "iters_max", "problems_gathered"):
        if k in line:
            out[k] = line[k]
    out.update(extra)
    print(json.dumps(out))
    comm.close()


def pcie_inclusive(ctx, a, xh, u0, stream):
    """steps x B problems as a host-memory caller sees them: H2D of the inputs, the solve, D2H of every
    problem's x, u and status (BASELINE.md section 3 counts host <-> device copies in wall time)."""
    B, N, dt = a.batch, a.N, 0.1
    ctx.synchronize()
    if not stream:
        tp = time.perf_counter()
        ctx.sqp_solve_batch(xh, u0, N, dt, a.method, with_trace=False)
        tp = time.perf_counter() - tp
        return {"value": B / tp, "unit": "solves/s", "ms_per_solve_batch": 1000.0 * tp,
                "note": "tmpc_sqp_solve_batch with host x/u (H2D, solve, D2H of x, u and the status arrays), one "
                        "batch, this GPU"}
    steps = a.steps
    P = B * steps
    xo = np.empty((P,) + xh.shape[1:])
    uo = np.empty((P,) + u0.shape[1:])
    st = np.empty((P, 4), dtype=np.int32)
    dxi, dui = ctx.alloc(xh.nbytes), ctx.alloc(u0.nbytes)
    sb = dict(x=ctx.alloc(xo.nbytes), u=ctx.alloc(uo.nbytes), st=ctx.alloc(st.nbytes))
    try:
        ctx.synchronize()
        tp = time.perf_counter()
        ctx.h2d(dxi, xh)
        ctx.h2d(dui, u0)
        ctx.solve_stream_device(solver_name(a), P, B, N, dt, dxi, dui, B, sb["x"], sb["u"], sb["st"])
        ctx.d2h(xo, sb["x"])
        ctx.d2h(uo, sb["u"])
        ctx.d2h(st, sb["st"])
        tp = time.perf_counter() - tp
    finally:
        for p in (dxi, dui, sb["x"], sb["u"], sb["st"]):
            ctx.free(p)
    return {"value": P / tp, "unit": "solves/s", "ms_per_step": 1000.0 * tp / steps,
            "note": f"{steps} x {B} problems with host inputs and outputs: H2D of x0 / u0 ({(xh.nbytes + u0.nbytes) / 1e6:.0f}"
                    f" MB), the stream, D2H of every problem's x, u and status ({(xo.nbytes + uo.nbytes + st.nbytes) / 1e6:.0f} MB, "
                    "pageable host memory); `value` is the HBM-resident rate"}


def line_args(a, **kw):
    import copy
    b = copy.copy(a)
    b.cost, b.erm, b.mpc_steps, b.pcg_warm_start, b.precision, b.solver = "quadratic", None, 0, False, "fp64", "sqp"
    b.method, b.limits, b.N, b.links = "PCG-SS", "none", 64, 6
    for k, v in kw.items():
        setattr(b, k, v)
    return b


# concurrent sub-streams per line (tmpc_stream.substreams), measured (profiles/r06/stream/probe_r06e.jsonl, 16
# copies): two overlap the latency-bound phases of config 3 / config 4 / the hard line by 3-5 %; the
# headline's k_qp fills every CU alone (no gain) and config 2's short iterations lose to the second stream
LINE_SUBSTREAMS = {"secondary": 2, "hard_limits": 2, "config3": 2, "config3_fp32": 2}


def run_config_lines(ctx, comm, rank, world, a):
    """The other BASELINE.json configurations beside the headline, each measured after it with its own
    timed region (barrier + synchronize, max over ranks), kernel table, roofline and parity sample:
      secondary    config 4: arm6 N = 64 SQP PCG-SS, soft torque + joint limits by augmented Lagrangian;
      hard_limits  the headline under hard ACTIVE_SET torque + velocity limits (the banded Schur path);
      config2      arm3 N = 32 SQP PCG-SS, B = 1024;
      config3      arm6 N = 64 iLQR, soft torque limits by augmented Lagrangian, fp64 and fp32 (BASELINE's
                   stated precision);
      config5      arm6 N = 128 receding-horizon MPC loop of 4 SQP PCG-SS horizon solves, mixed fp32
                   dynamics / fp64 PCG, PCG warm start, B = 8192."""
    out = {}
    lines = [
        ("secondary", line_args(a, limits="torque-joint-al"), a.secondary_steps, "config 4's per-GPU slice"),
        ("hard_limits", line_args(a, limits="torque-velocity-as"), a.hard_steps, "hard ACTIVE_SET limits"),
        ("config2", line_args(a, links=3, N=32, batch=1024), a.config_steps, "BASELINE config 2"),
        ("config3", line_args(a, solver="ilqr", limits="torque-al"), a.config_steps, "BASELINE config 3 (fp64)"),
        ("config3_fp32", line_args(a, solver="ilqr", limits="torque-al", precision="fp32"), a.config_steps,
         "BASELINE config 3 at its stated precision (fp32)"),
        ("config5", line_args(a, N=128, batch=8192, mpc_steps=4, precision="mixed", pcg_warm_start=True), 2,
         "BASELINE config 5's per-GPU slice"),
    ]
    for key, b, steps, label in lines:
        if key in a.skip_lines:
            continue
        stream = not a.lockstep and b.mpc_steps == 0
        b.substreams = LINE_SUBSTREAMS.get(key, 1)
        line, d, u0, counters, kernels, hb = run_line(ctx, comm, rank, world, b, steps, 1, stream,
                                                      a.lockstep_steps if stream else 0, b.substreams)
        nx, nu = 2 * b.links, b.links
        line["metric"] = f"MPC solves/sec (arm{b.links}.urdf, N={b.N}, {workload_name(b)}) -- {label}"
        if b.mpc_steps:
            line["metric"] = f"MPC horizon solves/sec (arm{b.links}.urdf, N={b.N}, {workload_name(b)}) -- {label}"
        line["config"] = line_config(b, world, workload_name(b))
        line["dtype"] = {"fp64": "f64", "fp32": "f32", "mixed": "f32 dynamics / f64 Schur-PCG"}[b.precision]
        line["roofline"] = line_roofline(b, b.N, nx, nu, kernels, counters, hb)
        line["value_basis"] = STREAM_BASIS if stream else "lock-step MPC loop: a step = 4 horizon solves of every problem"
        if rank == 0:
            line["parity"] = line_parity(ctx, key, b, d, u0)
        free_inputs(ctx, d)
        out[key] = line
        comm.barrier()
    setup_workload(ctx, a)
    return out


def _pool_map(fn, jobs):
    share, _, _ = host_cores()
    with mp.get_context("fork").Pool(max(1, min(share, len(jobs))), initializer=os.environ.__setitem__,
                                      initargs=("OMP_NUM_THREADS", "1")) as pool:
        return pool.map(fn, jobs, chunksize=1)


def _rel(x, y):
    return float(np.max(np.abs(np.asarray(x) - np.asarray(y)))) / max(1.0, float(np.max(np.abs(y))))


def line_parity(ctx, key, b, d, u0):
    """each line's parity sample on rank 0 (the GPU's lock-step batch solve of the same problems; the stream
    equals it per problem bitwise, stream_check):
      secondary   the oracle (oracle/sqp.py + oracle/soft.py) on the first --secondary-parity problems:
                  exit codes, SQP iterations, outer passes and per-QP PCG counts exact;
      hard_limits the oracle in the banded PCG's canonical order on the first --hard-parity problems, exact
                  integers; a problem whose run parts is replayed on the GPU's own inputs at the first
                  point the runs part (classify_hard_mismatch), and counts as unexplained otherwise;
      config2     the oracle on the first 64 problems, exact integers;
      config3     the committed oracle fixture (tests/golden/oracle_config3_arm6_N64_ilqr_al.npz, 8 problems):
                  exit codes, iterations, outer passes and alpha paths exact, x / u within 1e-5; at fp32 the
                  fixture's fp64 solves bound the deviation (parity unpinned: the reference is fp64 only);
      config5     the committed fp64 oracle MPC loop (oracle_config5_arm6_N128_mpc_sqp_pcgss.npz, 2 problems x
                  3 steps): per-step exit codes and SQP iterations exact, executed states within 1e-4."""
    n, N, B, dt = b.links, b.N, b.batch, 0.1
    nx = 2 * n
    if key in ("secondary", "hard_limits", "config2"):
        S = min(B, {"secondary": b.secondary_parity, "hard_limits": b.hard_parity, "config2": 64}[key])
        if S <= 0:
            return None
        fn = {"secondary": _cpu_solve_config4, "hard_limits": _cpu_solve_hard, "config2": _cpu_solve}[key]
        res = _pool_map(fn, [(b.seed0 + i, n, N) for i in range(S)])
        xh = x0_host(ctx, d["x0"], B, nx, N)[:S]
        if key == "secondary":
            ctx.set_soft_state(S, N)
        gr = ctx.sqp_solve_batch(xh, u0[:S], N, dt, b.method)
        par = parity_check(gr, res)
        if key == "secondary":
            soft_mism = [i for i, c in enumerate(res) if (int(gr["exit_soft"][i]), int(gr["outer_iter"][i]))
                         != (c["exit_soft"], c["outer_iter"])]
            par["mismatches"] += len([i for i in soft_mism if i not in par["mismatched_problems"]])
            par["compared"] += "; exit_soft, outer_iter (exact)"
        if key == "hard_limits":
            why = {i: classify_hard_mismatch(ctx, xh, u0[:S], N, dt, b.method, gr, i, res[i], b.limits)
                   for i in par["mismatched_problems"]}
            par["replayed"] = {str(i): w for i, w in why.items()}
            par["unexplained"] = sum(1 for w in why.values() if w["kind"] is None)
            par["mismatch_rate"] = par["mismatches"] / S
            par["note"] = HARD_PARITY_NOTE
        return par
    from oracle import sqp as osqp
    from trajoptmpcreference_amd.urdf import parse_urdf, planar_arm_urdf
    m = parse_urdf(planar_arm_urdf(n))
    if key in ("config3", "config3_fp32"):
        f = np.load(os.path.join(ROOT, "tests", "golden", "oracle_config3_arm6_N64_ilqr_al.npz"))
        xs, us = zip(*[osqp.initial_problem(m, N, dt, int(s)) for s in f["seeds"]])
        ctx.set_options(max_iter_softConstraints=int(f["max_iter_softConstraints"]),
                        max_iter_SQP_DDP=int(f["max_iter_SQP_DDP"]))
        ctx.set_soft_state(len(xs), N)
        try:
            r = ctx.ilqr_solve_batch(np.array(xs), np.array(us), N, dt)
        finally:
            ctx.set_options(max_iter_softConstraints=10, max_iter_SQP_DDP=100)
        cost = osqp.QuadCost(np.eye(nx), 100 * np.eye(nx), 0.1 * np.eye(n), np.zeros(nx))
        ints, alph, xerr, jerr = [], [], [], []
        for i in range(len(xs)):
            got = (int(r["exit_code"][i]), int(r["iter"][i]), int(r["exit_soft"][i]), int(r["outer_iter"][i]))
            ref = (int(f["exit_code"][i]), int(f["iter"][i]), int(f["exit_soft"][i]), int(f["outer_iter"][i]))
            ints.append(got == ref)
            al = f["alpha"][i]
            al = list(al[~np.isnan(al)])
            alph.append(list(r["trace"]["alpha"][i, 1:len(al) + 1]) == al)
            xerr.append(max(_rel(r["x"][i], f["x"][i]), _rel(r["u"][i], f["u"][i])))
            J = osqp.total_cost(cost, r["x"][i], r["u"][i], N)
            J64 = osqp.total_cost(cost, f["x"][i], f["u"][i], N)
            jerr.append(abs(J - J64) / abs(J64))
        out = {"checked": len(xs), "source": "tests/golden/oracle_config3_arm6_N64_ilqr_al.npz (oracle/ilqr.py)",
               "integers_identical": int(sum(ints)), "alpha_paths_identical": int(sum(alph)),
               "max_traj_rel_diff": max(xerr), "max_cost_rel_diff": max(jerr)}
        if key == "config3":
            out["mismatches"] = len(xs) - sum(a_ and b_ and e < 1e-5 for a_, b_, e in zip(ints, alph, xerr))
            out["compared"] = "exit code, iterations, exit_soft, outer_iter, alpha path (exact); x, u within 1e-5"
        else:
            out["compared"] = ("parity unpinned (no fp32 reference): deviation of the fp32 solves from the fp64 "
                               "oracle's; tests/test_gpu_precision.py bounds cost 1e-2, states 1e-1")
        return out
    if key == "config5":
        f = np.load(os.path.join(ROOT, "tests", "golden", "oracle_config5_arm6_N128_mpc_sqp_pcgss.npz"))
        steps = int(f["steps"])
        xs, us = zip(*[osqp.initial_problem(m, N, dt, int(s)) for s in f["seeds"]])
        r = ctx.mpc_batch(np.array(xs), np.array(us), N, dt, b.method, steps)
        ints = [list(r["exit_codes"][i]) == list(f["exit_codes"][i]) and list(r["iters"][i]) == list(f["iters"][i])
                for i in range(len(xs))]
        xerr = [_rel(r["x_exec"][i], f["x_exec"][i]) for i in range(len(xs))]
        return {"checked": len(xs), "steps": steps,
                "source": "tests/golden/oracle_config5_arm6_N128_mpc_sqp_pcgss.npz (oracle/mpc.py, fp64)",
                "mismatches": len(xs) - sum(ok and e < 1e-4 for ok, e in zip(ints, xerr)),
                "max_x_exec_rel_diff": max(xerr),
                "compared": "per-step exit codes and SQP iterations (exact); executed states within 1e-4 (mixed "
                            "precision against the fp64 oracle: parity unpinned for the floats)"}
    return None


HARD_PARITY_NOTE = (
    "oracle/sqp.py with oracle/hard.py's rows and pcg_canonical, the banded PCG's summation order.  replayed: each "
    "mismatched problem replayed on the GPU's own inputs at the first point the runs part (bench."
    "classify_hard_mismatch): 'pcg_count' -- the canonical-order PCG on the GPU's own S takes the GPU's count; "
    "'line_search' -- at the GPU's iterate the oracle's line search along the GPU's direction takes the GPU's "
    "outcome AND along the oracle's own direction (its own QP at that iterate) a different one: the step is "
    "decided by the two directions' rounding-amplified difference (direction_rel_diff), not by the line search")


def x0_host(ctx, d_x0, B, nx, N):
    x = np.empty((B, nx, N))
    ctx.d2h(x, d_x0)
    return x


if __name__ == "__main__":
    main()
