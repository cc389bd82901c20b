"""CPU-side checks of the C-ABI boundary: libtmpc.so loads (no GPU needed to
load it), exports every function include/tmpc.h declares, and the ctypes
binding covers exactly that set.  No compute calls are made here."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "tmpc.h")


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(tmpc_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_entry_points():
    fns = header_functions()
    for required in ["tmpc_create", "tmpc_destroy", "tmpc_last_error", "tmpc_set_model", "tmpc_set_cost_quadratic",
                     "tmpc_set_options", "tmpc_sqp_solve_batch", "tmpc_fd_batch", "tmpc_fd_grad_batch",
                     "tmpc_qp_batch", "tmpc_pcg_batch"]:
        assert required in fns


def test_library_exports_every_declared_symbol():
    from trajoptmpcreference_amd import _native
    lib = ctypes.CDLL(_native.LIB_PATH)
    missing = [f for f in header_functions() if not hasattr(lib, f)]
    assert not missing, missing


def test_binding_matches_header():
    from trajoptmpcreference_amd import _native
    assert sorted(_native.SIGNATURES) == header_functions()
    lib = _native.load_library()
    assert lib.tmpc_abi_version() == 10


def test_options_struct_layout_and_defaults():
    """tmpc_default_options is pure host code: the defaults are set_default_options'
    (TrajoptMPCReference.py:91-115)."""
    from trajoptmpcreference_amd import _native
    lib = _native.load_library()
    o = _native.tmpc_options()
    lib.tmpc_default_options(ctypes.byref(o))
    assert o.exit_tolerance_linSys == 1e-6 and o.max_iter_linSys == 100
    assert o.max_iter_SQP_DDP == 100 and o.exit_tolerance_SQP_DDP == 1e-6
    assert o.alpha_factor_SQP_DDP == 0.5 and o.alpha_min_SQP_DDP == 0.005
    assert o.rho_factor_SQP_DDP == 4 and o.rho_min_SQP_DDP == 1e-3 and o.rho_max_SQP_DDP == 1e3
    assert o.rho_init_SQP_DDP == 1e-3
    assert o.expected_reduction_min_SQP_DDP == 0.05 and o.expected_reduction_max_SQP_DDP == 3
    assert o.merit_mu == 10.0
    assert o.max_iter_softConstraints == 10 and o.exit_tolerance_softConstraints == 1e-6
    assert o.pcg_warm_start == 0   # the reference never forwards a PCG guess from SQP (:512-519)
    assert ctypes.sizeof(o) == 12 * 8 + 6 * 4   # 12 doubles, 6 int32, no padding


def test_box_limits_struct_size():
    from trajoptmpcreference_amd import _native
    # int32 mode[3] + reserved, double lb[3][8], ub[3][8], five double[3] option arrays
    assert ctypes.sizeof(_native.tmpc_box_limits) == 16 + 2 * 24 * 8 + 15 * 8


def test_null_context_is_an_error_not_a_crash():
    from trajoptmpcreference_amd import _native
    lib = _native.load_library()
    assert lib.tmpc_set_options(None, None) < 0
    assert lib.tmpc_last_error(None) == b"null context"


def test_trace_struct_layout():
    """tmpc_trace: 13 pointers in the header's order (ABI 6 added singular and hard_active)."""
    from trajoptmpcreference_amd import _native
    names = [f[0] for f in _native.tmpc_trace._fields_]
    assert names == ["iteration", "line_search_iteration", "alpha", "rho", "J", "c", "merit", "D", "reduction_ratio",
                     "succeeded_line_search", "pcg_iters", "singular", "hard_active"]
    assert ctypes.sizeof(_native.tmpc_trace) == 13 * 8


def test_stream_struct_layout():
    """tmpc_stream (ABI 10): four int32, five device pointers, then a tmpc_trace of device pointers."""
    from trajoptmpcreference_amd import _native
    names = [f[0] for f in _native.tmpc_stream._fields_]
    assert names == ["problems", "slots", "period", "substreams", "x_in", "u_in", "x_out", "u_out", "status", "trace"]
    assert ctypes.sizeof(_native.tmpc_stream) == 16 + 5 * 8 + 13 * 8


def test_stream_argument_errors_without_a_gpu():
    """the stream entry points validate before any device work: a null context fails, not crashes"""
    from trajoptmpcreference_amd import _native
    lib = _native.load_library()
    assert lib.tmpc_sqp_solve_stream_device(None, 8, 0.1, 4, None) < 0
    assert lib.tmpc_ilqr_solve_stream_device(None, 8, 0.1, None) < 0
