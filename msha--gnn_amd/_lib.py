"""ctypes binding of ``lib/libmsha_gnn.so`` (the C ABI in include/msha_gnn.h).

The library is the product path: there is no CPU or PyTorch fallback.  If it is
missing or fails to load, every op raises ``MshaLibraryError``.
"""
from __future__ import annotations

import ctypes as C
import os

import torch  # noqa: F401  (load torch's HIP runtime first: the library binds to it)

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MSHA_GNN_LIB", os.path.join(_PKG, "lib", "libmsha_gnn.so"))

ABI_VERSION = 16  # MSHA_ABI_VERSION of include/msha_gnn.h
MSHA_OK, MSHA_ERR_ARG, MSHA_ERR_UNSUPPORTED, MSHA_ERR_HIP = 0, -1, -2, -3


class MshaLibraryError(RuntimeError):
    pass


class MshaGraph(C.Structure):
    """Mirror of ``struct msha_graph`` (include/msha_gnn.h)."""

    _fields_ = [
        ("n_rows", C.c_int64), ("n_cols", C.c_int64), ("n_edges", C.c_int64),
        ("rowptr", C.c_void_p), ("col", C.c_void_p), ("rowflag", C.c_void_p),
        ("colptr", C.c_void_p), ("csc_row", C.c_void_p), ("csc_eid", C.c_void_p),
        ("n_chunks", C.c_int64), ("chunk_col", C.c_void_p), ("chunk_start", C.c_void_p),
        ("chunk_end", C.c_void_p),
        ("n_multi", C.c_int64), ("multi_col", C.c_void_p), ("multi_first", C.c_void_p),
        ("multi_count", C.c_void_p), ("csr_slot", C.c_void_p), ("rowmask", C.c_void_p),
    ]


P = C.c_void_p
I32, I64, U64, F32, SZ = C.c_int32, C.c_int64, C.c_uint64, C.c_float, C.c_size_t
GP = C.POINTER(MshaGraph)


class MshaGroups(C.Structure):
    """Mirror of ``struct msha_groups`` (include/msha_gnn.h)."""

    _fields_ = [("n_nodes", C.c_int64),
                ("gid3", C.c_void_p), ("gptr3", C.c_void_p), ("gmem3", C.c_void_p),
                ("gid4", C.c_void_p), ("gptr4", C.c_void_p), ("gmem4", C.c_void_p),
                ("max_group", C.c_int64)]


GRP = C.POINTER(MshaGroups)

HEAD_MAX_HEADS = 8


class MshaHeadParams(C.Structure):
    """Mirror of ``struct msha_head_params`` (include/msha_gnn.h)."""

    _fields_ = [("heads", C.c_int32), ("feat", C.c_int32), ("eps", C.c_float),
                ("momentum", C.c_float), ("slope", C.c_float)] + [
        (name, C.c_void_p * HEAD_MAX_HEADS)
        for name in ("u_weight", "u_bias", "u_running_mean", "u_running_var", "v_weight",
                     "v_bias", "v_running_mean", "v_running_var", "du_weight", "du_bias",
                     "dv_weight", "dv_bias")] + [
        ("num_batches_tracked", C.c_void_p * (2 * HEAD_MAX_HEADS))]


HPP = C.POINTER(MshaHeadParams)

MAX_SEGMENTS = 32
MAX_ADAM = 64


class MshaAdamTensor(C.Structure):
    """Mirror of ``struct msha_adam_tensor`` (include/msha_gnn.h)."""

    _fields_ = [("param", C.c_void_p), ("grad", C.c_void_p), ("exp_avg", C.c_void_p),
                ("exp_avg_sq", C.c_void_p), ("step", C.c_void_p), ("n", C.c_int64),
                ("dtype", C.c_int32), ("drop_p", C.c_float), ("drop_seed", C.c_uint64),
                ("drop_offset", C.c_uint64)]



class MshaSegment(C.Structure):
    """Mirror of ``struct msha_segment`` (include/msha_gnn.h)."""

    _fields_ = [("a", C.c_void_p), ("b", C.c_void_p), ("dst", C.c_void_p),
                ("rows", C.c_int64), ("cols", C.c_int64), ("lda", C.c_int64),
                ("ldb", C.c_int64), ("ldd", C.c_int64), ("p", C.c_float),
                ("seed", C.c_uint64), ("offset", C.c_uint64), ("a_dtype", C.c_int32),
                ("dst_dtype", C.c_int32)]

# name -> (restype, argtypes); every symbol here is declared in include/msha_gnn.h
SIGNATURES = {
    "msha_abi_version": (C.c_int, []),
    "msha_set_rng_counter": (C.c_int, [I32, P]),
    "msha_feed_step": (C.c_int, [P, P, I64, P, P]),
    "msha_ours_pack_draws": (I32, [I32]),
    "msha_wgrad_kernel": (I32, [I32]),
    "msha_get_rng_counter": (P, [I32]),
    "msha_last_error": (C.c_char_p, []),
    "msha_debug_timeline": (C.c_int, [P, I64]),
    "msha_debug_head_timeline": (C.c_int, [P]),
    "msha_debug_bip_timeline": (C.c_int, [P, I64]),
    "msha_dropout_keep_mask": (C.c_int, [U64, U64, I64, F32, P, P]),
    "msha_inter_adjacency": (C.c_int, [P, P, I64, I64, I64, P, P, P]),
    "msha_normalize_adjacency": (C.c_int, [P, I64, I64, P, P, P]),
    "msha_graph_workspace_size": (SZ, [I64, I64]),
    "msha_graph_rowmask": (C.c_int, [GP, P, P]),
    "msha_graph_count": (C.c_int, [P, I64, I64, P, P, P, P, SZ, P]),
    "msha_graph_fill": (C.c_int, [P, I64, I64, P, P, P, P, P, P, P, SZ, P]),
    "msha_edge_attention_supported": (C.c_int, [I32, I32]),
    "msha_edge_attention_fwd": (C.c_int, [GP, I32, I32, I32, P, P, P, F32, F32, U64, U64, P, P,
                                          P, P, P]),
    "msha_edge_attention_rowterms_preferred": (C.c_int, [GP, I32, I32, I32]),
    "msha_edge_attention_fwd_ex": (C.c_int, [GP, I32, I32, I32, P, P, P, F32, F32, U64, U64, P,
                                             P, P, P, P, P, P]),
    "msha_edge_attention_bwd_fused_ex": (C.c_int, [GP, I32, I32, I32, P, P, P, P, P, P, P, F32,
                                                   F32, U64, U64, P, P, P, P, P, P, P, SZ, P]),
    "msha_edge_attention_row_scores_supported": (C.c_int, [GP, I32, I32, I32]),
    "msha_edge_attention_row_scores_preferred": (C.c_int, [GP, I32, I32, I32]),
    "msha_edge_attention_fwd_rs": (C.c_int, [GP, I32, I32, I32, P, P, P, F32, F32, U64, U64, P,
                                             P, P, P, P, P]),
    "msha_edge_attention_bwd_fused_rs": (C.c_int, [GP, I32, I32, I32, P, P, P, P, P, P, P, F32,
                                                   F32, U64, U64, P, P, P, P, P, P, P, SZ, P]),
    "msha_edge_attention_bwd_rows": (C.c_int, [GP, I32, I32, I32, P, P, P, P, P, P, P, P, P, P,
                                               F32, F32, U64, U64, P, P, P, I32, P, P]),
    "msha_edge_attention_bwd_fused_workspace_size": (SZ, [GP, I32, I32]),
    "msha_edge_attention_bwd_fused": (C.c_int, [GP, I32, I32, I32, P, P, P, P, P, P, P, F32,
                                                F32, U64, U64, P, P, P, P, P, SZ, P]),
    "msha_bip_supported": (C.c_int, [GP, I32, I32, I32]),
    "msha_bip_workspace_size": (SZ, [GP, I32, I32]),
    "msha_bip_attention_fwd": (C.c_int, [GP, I32, I32, I32, P, P, P, P, F32, F32, U64, U64, P,
                                         P, P, P, P, P, SZ, P]),
    "msha_bip_attention_bwd": (C.c_int, [GP, I32, I32, I32, P, P, P, P, P, P, P, P, F32, F32,
                                         U64, U64, P, P, P, P, P, SZ, P]),
    "msha_csc_aggregate_workspace_size": (SZ, [GP, I32, I32]),
    "msha_csc_aggregate": (C.c_int, [GP, I32, I32, I32, P, P, I32, P, P, P, P, SZ, P]),
    "msha_gal_fwd": (C.c_int, [GP, P, F32, U64, U64, P, P]),
    "msha_gal_bwd": (C.c_int, [GP, P, P, F32, U64, U64, P, P]),
    "msha_gemm_workspace_size": (SZ, [I64, I64, I32]),
    "msha_gemm_f32": (C.c_int, [I64, I64, I64, P, I64, I64, P, I64, I64, P, I64, F32, I32, P, SZ,
                                P]),
    "msha_project_scores": (C.c_int, [I64, I64, I32, I32, P, P, P, P, P, P, P, P]),
    "msha_project_scores_row_order": (C.c_int, [I64, I64, I32, I32, I32]),
    "msha_gemm_f32_head_outer": (C.c_int, [I64, I64, I64, P, I64, I64, P, I64, I64, P, I64, F32,
                                           I32, P, SZ, I32, I32, I32, P, P, P, P, P]),
    "msha_head_outer_colsum_workspace_size": (SZ, [I64]),
    "msha_gemm_f32_head_outer_colsum": (C.c_int, [I64, I64, I64, P, I64, I64, P, I64, I64, P,
                                                  I64, I32, P, SZ, I32, I32, P, P, P, P, P, P,
                                                  P, P, SZ, P]),
    "msha_gemm_f32_head_outer_colsum_w": (C.c_int, [I64, I64, I64, P, I64, I64, P, I64, I64, P,
                                                    I64, I32, P, SZ, I32, I32, P, P, P, P, P,
                                                    I64, P, P, P, SZ, P]),
    "msha_add_head_outer": (C.c_int, [I64, I32, I32, P, P, P, P, P, P, P]),
    "msha_head_colsum_workspace_size": (SZ, [I64, I32, I32]),
    "msha_head_colsum": (C.c_int, [I64, I32, I32, I32, P, P, P, P, P, P, SZ, P]),
    "msha_gemm_bf16_workspace_size": (SZ, [I64, I64, I32]),
    "msha_gemm_bf16": (C.c_int, [I64, I64, I64, P, I64, I64, P, I64, I64, P, I64, I32, I32, P, SZ,
                                 I32, I32, I32, P, P, P, P, P]),
    "msha_project_scores_bf16": (C.c_int, [I64, I64, I32, I32, P, P, P, P, P, P, P, P]),
    "msha_bn_workspace_size": (SZ, [I64, I32]),
    "msha_bn_lrelu_fwd": (C.c_int, [I64, I32, I32, P, P, P, F32, F32, I32, F32, P, P, P, P, P, P,
                                    SZ, P]),
    "msha_bn_lrelu_bwd": (C.c_int, [I64, I32, I32, P, P, P, P, P, P, F32, P, P, P, P, SZ, P]),
    "msha_pair_linear": (C.c_int, [I64, I64, I64, P, I64, P, P, I64, P, I64, I64, P, P, I32, F32,
                                   U64, U64, P, P]),
    "msha_pair_inner_fwd": (C.c_int, [I64, I32, P, I64, P, P, I64, P, P, P]),
    "msha_pair_inner_fwd_bf16": (C.c_int, [I64, I32, P, I64, P, P, I64, P, P, P]),
    "msha_pair_inner_fwd_ex": (C.c_int, [I64, I32, I32, P, I64, P, I64, P, I64, P, I64, P, P,
                                         P]),
    "msha_bip2_bwd_min_rows": (I64, [I64]),
    "msha_pair_index_check": (C.c_int, [I64, P, I64, P, I64, P, P]),
    "msha_pair_linear_bf16": (C.c_int, [I64, I64, I64, P, I64, P, P, I64, P, P, P, I32, F32, U64,
                                        U64, P, P]),
    "msha_pair_linear_bf16_ex": (C.c_int, [I64, I64, I64, P, I64, P, P, I64, P, P, P, I32, F32,
                                           U64, U64, I32, P, P]),
    "msha_pair_inner_bwd": (C.c_int, [I64, I32, P, I64, P, P, I64, P, P, P, P, P, P]),
    "msha_pair_mlp_dz": (C.c_int, [I64, P, P, F32, I32, P, P]),
    "msha_pair_hadamard": (C.c_int, [I64, I32, P, I64, P, P, I64, P, P, P, P, P]),
    "msha_pair_hadamard_sigmoid": (C.c_int, [I64, I32, P, I64, P, P, I64, P, P, P, P, P, P]),
    "msha_ours_intra_fwd": (C.c_int, [GP, GRP, I64, P, I32, I32, I32, P, P, P, P, P, P, P, F32, F32,
                                      U64, U64, P, P, P]),
    "msha_ours_workspace_size": (SZ, [GRP, I64, I32, I32]),
    "msha_ours_intra_bwd": (C.c_int, [GP, GRP, I64, P, I32, I32, I32, P, P, P, P, P, I32, F32, F32,
                                      U64, U64, P, P, P, P, P, P, P, SZ, P]),
    "msha_segments": (C.c_int, [I32, P, P]),
    "msha_adam_workspace_size": (SZ, []),
    "msha_adam_step": (C.c_int, [I32, P, C.c_double, C.c_double, C.c_double, C.c_double,
                                 C.c_double, P, P]),
    "msha_project_small_supported": (C.c_int, [I64, I64, I32, I32]),
    "msha_project_small": (C.c_int, [I64, I64, I32, I32, P, P, P, P, P, P, P, P]),
    "msha_project_small_bwd": (C.c_int, [I64, I64, I32, I32, P, P, P, P, P, P, P, P, P, P, P, P,
                                         P]),
    "msha_dropout_keep_mask4": (C.c_int, [U64, U64, I64, F32, P, P]),
    "msha_dropout_keep_mask_word": (C.c_int, [U64, U64, I64, F32, I32, P, P]),
    "msha_nll_rows_fwd": (C.c_int, [I64, I64, I64, P, P, I32, P, I64, P, P]),
    "msha_nll_rows_bwd": (C.c_int, [I64, I64, I64, P, P, P, I32, P, I64, P]),
    "msha_head_supported": (C.c_int, [I64, I32, I32]),
    "msha_head_workspace_size": (SZ, [GP, I32, I32]),
    "msha_head_fwd": (C.c_int, [GP, HPP, I32, P, P, P, I32, F32, U64, F32, U64, P, P, P, SZ, P]),
    "msha_head_bwd": (C.c_int, [GP, HPP, I32, P, P, P, F32, U64, F32, U64, P, P, P, P, P, P, I64,
                                P, SZ, P]),
    "msha_bip_defer_reduce": (C.c_int, [I32]),
    "msha_nll_rows_bwd_flags": (C.c_int, [I64, I64, I64, P, P, P, I32, P, I64, P, P, P]),
    "msha_head_bwd_flagged": (C.c_int, [GP, HPP, I32, P, P, P, F32, U64, F32, U64, P, P, P, P, P,
                                        P, P, P, I64, P, SZ, P]),
}

_lib = None
_load_error = None


def load(path: str = LIB_PATH):
    """Load (once) and type the library.  Raises MshaLibraryError if unavailable."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        _load_error = (f"HIP library not found at {path}; build it with "
                       f"`python msha--gnn_amd/build.py` (or __graft_entry__.build())")
        raise MshaLibraryError(_load_error)
    try:
        lib = C.CDLL(path)
    except OSError as e:  # pragma: no cover - depends on the box
        _load_error = f"failed to load {path}: {e}"
        raise MshaLibraryError(_load_error) from e
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.msha_abi_version() != ABI_VERSION:
        raise MshaLibraryError("ABI version mismatch")
    _lib = lib
    return lib


def available() -> bool:
    try:
        load()
        return True
    except MshaLibraryError:
        return False


def exported_symbols():
    return sorted(SIGNATURES)


def raise_for(rc: int, name: str):
    """Raise the library's thread-local message for a failed call."""
    msg = load().msha_last_error().decode(errors="replace")
    raise RuntimeError(f"{name} failed ({rc}): {msg}")


_FNS: dict = {}  # name -> typed ctypes function (one getattr per name)


def fn(name: str):
    f = _FNS.get(name)
    if f is None:
        f = _FNS[name] = getattr(load(), name)
    return f


def call(name: str, *args):
    """Invoke an ABI function; raise on a non-zero status with the library message."""
    f = _FNS.get(name)
    if f is None:
        f = fn(name)
    rc = f(*args)
    if rc != MSHA_OK:
        raise_for(rc, name)
    return rc


def ptr(t) -> int | None:
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return t.data_ptr()


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_handle(device=None) -> int:
    """The current HIP stream of ``device`` (torch.device, index or None = current) as
    an integer handle -- the raw-stream query, without building a torch Stream object
    per call (the ops issue one per launch)."""
    if _raw_stream is not None:
        if device is None:
            idx = torch.cuda.current_device()
        elif isinstance(device, int):
            idx = device
        else:
            if isinstance(device, str):
                device = torch.device(device)
            idx = device.index if device.index is not None else torch.cuda.current_device()
        return _raw_stream(idx)
    return torch.cuda.current_stream(device).cuda_stream


def require_cuda(*tensors):
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise RuntimeError("msha_gnn_amd ops run on the GPU only (got a CPU tensor); "
                               "move the model and adjacency to the HIP device")
