"""ctypes binding of libhichap_hip.so (the C-ABI declared in
include/hichap_hip.h).

The shared library is built in-tree by ``__graft_entry__.build()`` (or
``make -C hichap_master_amd/csrc``).  There is no CPU fallback: if the library
is missing or no GPU is visible, every compute entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# HH_LIB: another build of the library (build experiments, e.g. -DHH_KWBITS=12)
LIB_PATH = os.environ.get("HH_LIB") or os.path.join(_HERE, "libhichap_hip.so")

HH_OK = 0


class HipLibraryError(RuntimeError):
    """Raised when the HIP library is missing or a C-ABI call fails."""

    def __init__(self, code, msg):
        super().__init__(f"[hh rc={code}] {msg}")
        self.code = code


class MatrixInfo(C.Structure):
    _fields_ = [(n, C.c_int64) for n in (
        "n_bins", "row_lo", "row_hi", "nnz_upper", "n_entries", "n_slots", "n_tiles",
        "n_units", "n_wide", "device_bytes", "n_slots_narrow", "payload_bytes")] + [
        (n, C.c_int32) for n in ("n_chroms", "ignore_diags", "cis_only", "device", "band_w", "n_units_flat")] + [
        ("n_band", C.c_int64), ("payload_bytes_flat", C.c_int64)] + [
        (n, C.c_int32) for n in ("band_w4", "upper")]


class SynthParams(C.Structure):
    _fields_ = [
        ("n_chroms", C.c_int32), ("chrom_nbins", C.POINTER(C.c_int32)),
        ("A", C.c_double), ("decay", C.c_double), ("comp_strength", C.c_double),
        ("vis_sigma", C.c_double), ("gap_frac", C.c_double), ("trans_density", C.c_double),
        ("comp_block", C.c_int32), ("ignore_diags", C.c_int32), ("cis_only", C.c_int32),
        ("pad_", C.c_int32), ("seed", C.c_uint64)]


class IceOpts(C.Structure):
    _fields_ = [
        ("mad_max", C.c_int32), ("min_nnz", C.c_int32), ("min_count", C.c_double),
        ("tol", C.c_double), ("max_iters", C.c_int32), ("rescale_marginals", C.c_int32),
        ("check_every", C.c_int32), ("pad_", C.c_int32)]


P = C.c_void_p
I32, I64, F64 = C.c_int32, C.c_int64, C.c_double
PI32, PI64, PF64 = C.POINTER(C.c_int32), C.POINTER(C.c_int64), C.POINTER(C.c_double)

# name -> (restype, argtypes); every function returns int status unless noted
SIGNATURES = {
    "hh_last_error": (C.c_char_p, []),
    "hh_version": (C.c_int, []),
    "hh_device_count": (C.c_int, [PI32]),
    "hh_set_device": (C.c_int, [I32]),
    "hh_synchronize": (C.c_int, [P]),
    "hh_device_copy": (C.c_int, [P, P, I64, P]),
    "hh_tune": (C.c_int, [C.c_char_p, I64]),
    "hh_ktime_enable": (C.c_int, [I32]),
    "hh_ktime_query": (C.c_int, [C.c_char_p, P, P]),
    "hh_ktime_reset": (C.c_int, []),
    "hh_matrix_from_pixels": (C.c_int, [P, P, P, I64, I64, P, I32, I32, I32, I64, I64, P, C.POINTER(P)]),
    "hh_matrix_from_pixels_device": (C.c_int, [P, P, P, I64, I64, P, I32, I32, I32, I64, I64, P, C.POINTER(P)]),
    "hh_matrix_free": (C.c_int, [P]),
    "hh_matrix_get_info": (C.c_int, [P, C.POINTER(MatrixInfo)]),
    "hh_matrix_export_upper": (C.c_int, [P, P, P, P, PI64]),
    "hh_synth_count": (C.c_int, [C.POINTER(SynthParams), P, P, P]),
    "hh_synth_build": (C.c_int, [C.POINTER(SynthParams), I64, I64, P, C.POINTER(P)]),
    "hh_synth_dense": (C.c_int, [P, I32, P, P]),
    "hh_synth_pixels": (C.c_int, [C.POINTER(SynthParams), I32, P, C.POINTER(P)]),
    "hh_pixels_get": (C.c_int, [P, P, P, P, PI64]),
    "hh_pixels_free": (C.c_int, [P]),
    "hh_ice_balance": (C.c_int, [P, C.POINTER(IceOpts), P, P, P, P, P, PF64, P]),
    "hh_ice_create": (C.c_int, [P, C.POINTER(IceOpts), C.POINTER(P)]),
    "hh_ice_free": (C.c_int, [P]),
    "hh_ice_n_groups": (C.c_int, [P, PI32]),
    "hh_ice_marg_local": (C.c_int, [P, I32, P, P]),
    "hh_ice_set_marg": (C.c_int, [P, P, I32, I64, P, P]),
    "hh_ice_filter_nnz": (C.c_int, [P, P]),
    "hh_ice_filter_count_mad": (C.c_int, [P, P]),
    "hh_ice_update": (C.c_int, [P, P]),
    "hh_ice_active_groups": (C.c_int, [P, PI32, P]),
    "hh_ice_iterations_done": (C.c_int, [P, PI32]),
    "hh_ice_run": (C.c_int, [P, I32, P]),
    "hh_ice_finalize": (C.c_int, [P, P, P, P, P, P, P]),
    "hh_ice_last_sweep_timing": (C.c_int, [P, PF64, PI32, PF64]),
    "hh_ice_swept_bytes": (C.c_int, [P, PI64]),
    "hh_ice_get_bias": (C.c_int, [P, P, P]),
    "hh_sweep_trace": (C.c_int, [P, I64, PI64]),
    "hh_matrix_stream_probe": (C.c_int, [P, I32, PF64, I32]),
    "hh_comm_unique_id": (C.c_int, [P]),
    "hh_comm_init": (C.c_int, [P, I32, I32, C.POINTER(P)]),
    "hh_comm_free": (C.c_int, [P]),
    "hh_comm_allgather": (C.c_int, [P, I64, P, P, P]),
    "hh_comm_reduce_scatter": (C.c_int, [P, I64, P, P, P]),
    "hh_ice_set_column_exchange": (C.c_int, [P, I32, I32, P, P, P, P, P]),
    "hh_ice_balance_sharded": (C.c_int, [P, C.POINTER(IceOpts), I32, I32, P, P, P, P, P, P, P, P, PF64, P]),
    "hh_ice_balance_cis_local": (C.c_int, [P, C.POINTER(IceOpts), I32, I64, P, P, P, P, P, P, P, PF64, P]),
    "hh_ice_filters_sharded": (C.c_int, [P, I32, P, P, P, P]),
    "hh_ice_run_sharded": (C.c_int, [P, I32, P, P, P, I32, P]),
    "hh_dense_rowstats": (C.c_int, [P, I32, I64, P, P, P, P, I32, P]),
    "hh_dense_symvc": (C.c_int, [P, I32, I64, P, P, F64, F64, P, I32, P]),
    "hh_twostep": (C.c_int, [P, P, P, I64, P, P, P, P, I32, P]),
    "hh_twostep_batch": (C.c_int, [I32, P, P, P, P, P, P, P, P, I32, P]),
    "hh_dense_from_cells": (C.c_int, [P, P, P, I64, I64, I64, I32, I32, P, P]),
    "hh_dense_upper_count": (C.c_int, [P, I64, PI64, P]),
    "hh_dense_upper_write": (C.c_int, [P, I64, P, P, P, P]),
    "hh_comp_create": (C.c_int, [P, I64, I32, P, C.POINTER(P)]),
    "hh_comp_free": (C.c_int, [P]),
    "hh_comp_colnnz": (C.c_int, [P, P, P]),
    "hh_comp_diag_sums": (C.c_int, [P, P, P, P]),
    "hh_comp_sliding_oe": (C.c_int, [P, P, I32, P]),
    "hh_comp_get_sliding_oe": (C.c_int, [P, P, P]),
    "hh_comp_correlation": (C.c_int, [P, P, P, I64, P]),
    "hh_comp_get_cor": (C.c_int, [P, P, P]),
    "hh_comp_set_cor": (C.c_int, [P, P, P]),
    "hh_gap_scan": (C.c_int, [P, I64, I32, I32, P, I32, P]),
    "hh_di_scan": (C.c_int, [P, I64, I32, P, P, I32, P, I32, P]),
    "hh_band_from_pixels": (C.c_int, [P, P, P, I64, P, I64, I64, I64, I32, P, I32, P]),
    "hh_tad_scan_pixels": (C.c_int, [P, P, P, I64, P, I64, I64, I64, I32, P, I32, P, P, I32, P]),
    "hh_viterbi_gmm": (C.c_int, [P, I64, I32, I32, P, P, P, P, P, P, P]),
    "hh_comp_pca": (C.c_int, [P, I32, F64, I32, P, P, P, P]),
    "hh_comp_select_stats": (C.c_int, [P, P, I32, F64, P, P]),
    "hh_comp_pca_status": (C.c_int, [P, PI32, PI32, PI32, PI32]),
    "hh_sym_topk": (C.c_int, [P, I32, I32, P, P]),
    "hh_binner_create": (C.c_int, [I32, C.c_char_p, P, I32, I32, C.POINTER(P)]),
    "hh_binner_free": (C.c_int, [P]),
    "hh_binner_add_target": (C.c_int, [P, I32, I32, P, P, I64, PI32]),
    "hh_binner_feed": (C.c_int, [P, C.c_char_p, I64, P, I64, P]),
    "hh_binner_add_impute_target": (C.c_int, [P, I32, I32, P, P, I64, P, I32, I64, F64, PI32]),
    "hh_binner_last_reached": (C.c_int, [P, PI64, PI32]),
    "hh_binner_set_stale": (C.c_int, [P, I32, I64, I32]),
    "hh_binner_feed_device": (C.c_int, [P, P, I64, P, P]),
    "hh_binner_stats": (C.c_int, [P, P]),
    "hh_binner_finish": (C.c_int, [P, P]),
    "hh_binner_target_nnz": (C.c_int, [P, I32, PI64, PI64]),
    "hh_binner_download": (C.c_int, [P, I32, P, P, P]),
    "hh_binner_pixels_device": (C.c_int, [P, I32, P, P, P]),
    "hh_gw_create": (C.c_int, [P, P, P, I64, P, P, P, I64, I64, P, I32, P, C.POINTER(P)]),
    "hh_gw_create_device": (C.c_int, [P, P, P, I64, P, P, P, I64, I64, P, I32, P, C.POINTER(P)]),
    "hh_gw_free": (C.c_int, [P]),
    "hh_gw_stats": (C.c_int, [P, P, P, P, PI64]),
    "hh_gw_alpha": (C.c_int, [P, P, P]),
    "hh_gw_correct": (C.c_int, [P, P, F64, PI64, P]),
    "hh_gw_correct_count": (C.c_int, [P, P, F64, PI64, P]),
    "hh_gw_correct_write": (C.c_int, [P, P, P, P, P]),
    "hh_gw_result": (C.c_int, [P, P, P, P, P]),
    "hh_gw_result_device": (C.c_int, [P, P, P, P]),
    "hh_hiccups_create": (C.c_int, [P, P, P, I64, I32, I32, I32, P, C.POINTER(P)]),
    "hh_hiccups_free": (C.c_int, [P]),
    "hh_hiccups_set_pixels": (C.c_int, [P, P, P, I64, P]),
    "hh_hiccups_width": (C.c_int, [P, I32, PI64, P]),
    "hh_hiccups_reset": (C.c_int, [P, P]),
    "hh_hiccups_results": (C.c_int, [P, P, P, P, P, P, P]),
    "hh_synth_pairs_text": (C.c_int, [I32, C.c_char_p, P, I64, F64, F64, I32, C.c_uint64, I64, P, I64, PI64, P]),
}

_lib = None


def load(path: str = LIB_PATH):
    """Load the shared library and declare every signature (fails loudly)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise HipLibraryError(-100, f"{path} not built; run __graft_entry__.build() "
                                    f"or `make -C hichap_master_amd/csrc`")
    # torch-ROCm ships its own HIP runtime with the same SONAME as /opt/rocm's
    # (libamdhip64.so.7).  Importing torch first makes that runtime the
    # process's only one, so torch streams/allocations and this library agree.
    try:
        import torch  # noqa: F401
    except Exception:
        pass
    lib = C.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    # measurement knobs for a whole process (A/B runs of tests and benches):
    # HH_TUNE="key=value,key=value" -> hh_tune at load
    for kv in filter(None, os.environ.get("HH_TUNE", "").split(",")):
        k, v = kv.split("=")
        call("hh_tune", k.strip().encode(), int(v))
    return lib


def call(name, *args):
    """Call a status-returning entry point; raise on failure."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != HH_OK:
        msg = lib.hh_last_error().decode(errors="replace")
        raise HipLibraryError(rc, f"{name}: {msg}")
    return rc


def ptr(a):
    """Raw pointer of a NumPy array or torch tensor (None -> NULL)."""
    if a is None:
        return None
    if hasattr(a, "data_ptr"):
        return C.c_void_p(a.data_ptr())
    return a.ctypes.data_as(C.c_void_p)


def ktime(name: str):
    """(total_ms, calls) of one kernel name recorded since hh_ktime_reset
    while hh_ktime_enable(1) was on (measurement only)."""
    t = C.c_double(0.0)
    n = C.c_int64(0)
    call("hh_ktime_query", name.encode(), C.byref(t), C.byref(n))
    return t.value, n.value


def device_count() -> int:
    n = C.c_int32(0)
    try:
        call("hh_device_count", C.byref(n))
    except HipLibraryError:
        return 0
    return int(n.value)


_have_gpu = False


def require_gpu():
    """Raise unless a HIP device is visible (cached once found: the runtime's
    device query costs ~1 ms)."""
    global _have_gpu
    if _have_gpu:
        return
    if device_count() < 1:
        raise HipLibraryError(-101, "no HIP device visible: the HIP path has no CPU fallback")
    _have_gpu = True
