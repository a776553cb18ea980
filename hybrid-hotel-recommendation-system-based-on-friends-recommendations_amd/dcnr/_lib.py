"""ctypes binding of libdcnr.so (C ABI declared in include/dcnr.h).

The library is loaded after ``torch`` so that its ``libamdhip64.so.7``
dependency binds to the HIP runtime torch already loaded (one runtime, one
set of streams).  There is no fallback: if the library is missing the import
of any compute entry point raises.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must precede the HIP library load)

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("DCNR_LIB", os.path.join(PKG_ROOT, "lib", "libdcnr.so"))

DCNR_OK, DCNR_BAD_ARG, DCNR_INDEX_OOB, DCNR_HIP_ERROR, DCNR_UNSUPPORTED_SHAPE, \
    DCNR_WORKSPACE_TOO_SMALL = range(6)
PREC_FP32, PREC_BF16 = 0, 1
EVAL, TRAIN = 0, 1
FLAG_CHECK_INDICES = 1
FLAG_KEEP_INTERMEDIATES = 2
FLAG_FUSED_TOWER = 4
FLAG_ROW_MAP = 8
ABI_VERSION = 4
# dcnr_ws_tensor (include/dcnr.h)
WS_KINDS = ["x0", "h", "t1", "t2", "a1", "mask_a1", "mask_h", "bn_mean", "bn_invstd", "bn_scale",
            "bn_shift", "du", "dt2", "da", "dt1", "G", "dx0", "zc", "xcoef", "sc", "row_map"]

ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64,
                                ctypes.c_void_p)
# dcnr_grad_ready_fn(ctx, group, stream); groups below
GRAD_READY_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p)
GRADS_DENSE, GRADS_EMBEDDING = 0, 1
TOUCHED_MAX_WORLD = 64   # DCNR_TOUCHED_MAX_WORLD: ranks dcnr_emb_touched_rows counts owners for


class ModelDesc(ctypes.Structure):
    _fields_ = [
        ("n_users", ctypes.c_int64),
        ("n_items", ctypes.c_int64),
        ("n_cat", ctypes.c_int32),
        ("cat_rows", ctypes.POINTER(ctypes.c_int64)),
        ("emb_dim", ctypes.c_int32),
        ("n_num", ctypes.c_int32),
        ("hidden", ctypes.c_int32),
        ("n_cross", ctypes.c_int32),
        ("n_res", ctypes.c_int32),
        ("dropout", ctypes.c_float),
        ("precision", ctypes.c_int32),
        ("flags", ctypes.c_uint32),
        ("bn_allreduce", ALLREDUCE_FN),
        ("bn_allreduce_ctx", ctypes.c_void_p),
        ("grad_ready", GRAD_READY_FN),
        ("grad_ready_ctx", ctypes.c_void_p),
        ("error_mirror", ctypes.c_void_p),
    ]


# exported symbol -> (restype, argtypes); must match include/dcnr.h
_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_SIGS = {
    "dcnr_abi_version": (ctypes.c_int, []),
    "dcnr_last_error": (ctypes.c_char_p, []),
    "dcnr_input_dim": (_I64, [ctypes.POINTER(ModelDesc)]),
    "dcnr_workspace_size": (ctypes.c_int, [ctypes.POINTER(ModelDesc), _I64, ctypes.c_int,
                                           ctypes.POINTER(ctypes.c_size_t)]),
    "dcnr_workspace_offset": (ctypes.c_int, [ctypes.POINTER(ModelDesc), _I64, ctypes.c_int,
                                             ctypes.c_int, ctypes.c_int, ctypes.POINTER(_I64)]),
    "dcnr_forward": (ctypes.c_int, [ctypes.POINTER(ModelDesc), _P, _P, _P, _P, _P, _I64,
                                    ctypes.c_int, ctypes.c_uint64, _P, _P, ctypes.c_size_t, _P]),
    "dcnr_gather_cross": (ctypes.c_int, [ctypes.POINTER(ModelDesc), _P, _P, _P, _P, _P, _I64, _P,
                                         _I64, _P, _I64, _P, _P]),
    "dcnr_backward": (ctypes.c_int, [ctypes.POINTER(ModelDesc), _P, _P, _P, _P, _P, _P, _I64, _P,
                                     ctypes.c_uint64, ctypes.c_int, _P, ctypes.c_size_t, _P]),
    "dcnr_emb_touched_rows": (ctypes.c_int, [ctypes.POINTER(ModelDesc), _P, ctypes.c_size_t, _I64,
                                             ctypes.c_int32, _P, _P, _I64, ctypes.c_int32, _P, _P,
                                             _P, _P]),
    "dcnr_sparse_pack": (ctypes.c_int, [_P, _P, _I64, _P, ctypes.c_int32, ctypes.c_int32, _P, _P, _P]),
    "dcnr_sparse_accumulate": (ctypes.c_int, [_P, _I64, _I64, ctypes.c_int32, _P, _P, _P,
                                              ctypes.c_int32, _P]),
    "dcnr_bce_workspace_size": (ctypes.c_size_t, []),
    "dcnr_bce_with_logits": (ctypes.c_int, [_P, _P, _I64, _P, _P, ctypes.c_float, _P,
                                            ctypes.c_size_t, _P]),
    "dcnr_adam_step": (ctypes.c_int, [ctypes.c_int32, _P, _P, _P, _P, _P, ctypes.c_float,
                                      ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                      ctypes.c_float, _I64, ctypes.c_int, _P]),
    "dcnr_adam_step_rows": (ctypes.c_int, [ctypes.c_int32, _P, _P, _P, _P, _P, _P, _P,
                                           ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                           ctypes.c_float, ctypes.c_float, _I64, ctypes.c_int, _P]),
    "dcnr_row_inv_norms": (ctypes.c_int, [_P, _I64, ctypes.c_int32, _P, _P]),
    "dcnr_cosine_topk_workspace_size": (ctypes.c_size_t, [_I64, _I64, ctypes.c_int32]),
    "dcnr_cosine_topk": (ctypes.c_int, [_P, _P, _I64, ctypes.c_int32, _P, _I64, ctypes.c_int32,
                                        _P, _P, _P, ctypes.c_size_t, _P]),
    "dcnr_cosine_pack_rows": (ctypes.c_int, [_P, _P, _I64, ctypes.c_int32, _P, _P]),
    "dcnr_cosine_topk_packed": (ctypes.c_int, [_P, _P, _P, _I64, ctypes.c_int32, _P, _I64,
                                               ctypes.c_int32, _P, _P, _P, ctypes.c_size_t, _P]),
    "dcnr_topk_merge": (ctypes.c_int, [_P, _P, ctypes.c_int32, _I64, ctypes.c_int32, _P, _P, _P]),
    "dcnr_gather_rows": (ctypes.c_int, [_P, _I64, _I64, ctypes.c_int32, _P, _P, _P, _P]),
    "dcnr_candidate_union": (ctypes.c_int, [_P, _I64, _P, ctypes.c_int32, _P, _P, _P]),
    "dcnr_ranking_batch": (ctypes.c_int, [_P, _I64, _I64, _P, ctypes.c_int32, _P, ctypes.c_int32,
                                          _I64, _P, _P, _P, _P, _P]),
    "dcnr_rank_by_score": (ctypes.c_int, [_P, _I64, _P, _P]),
    "dcnr_mmr_rerank": (ctypes.c_int, [_P, _P, ctypes.c_int32, _P, _P, _I64, ctypes.c_float,
                                       ctypes.c_int32, _P, _P, _P]),
    "dcnr_check_errors": (ctypes.c_int, [_P, ctypes.c_size_t, _P]),
    "dcnr_linear_bf16": (ctypes.c_int, [_P, _I64, _I64, ctypes.c_int32, _P, _I64, ctypes.c_int32,
                                        _P, _P, _I64, ctypes.c_int, _P]),
    "dcnr_linear_wgrad_workspace_size": (ctypes.c_size_t, [ctypes.c_int32, ctypes.c_int32, _I64]),
    "dcnr_linear_wgrad_bf16": (ctypes.c_int, [_P, _I64, _P, _I64, _I64, ctypes.c_int32,
                                              ctypes.c_int32, _P, ctypes.c_int, _P,
                                              ctypes.c_size_t, _P]),
    "dcnr_profile_enable": (None, [ctypes.c_int]),
    "dcnr_profile_collect": (ctypes.c_int, [_P, _P, ctypes.c_int32]),
    "dcnr_profile_collect_bytes": (ctypes.c_int, [_P, _P, _P, ctypes.c_int32]),
}

KERNEL_CLASSES = ["gather_cross", "gemm_fwd", "gemm_dx", "gemm_dw", "rowwise", "reduce",
                  "cross_bwd", "head", "adam", "knn", "pack", "serve", "emb_sort", "emb_sum",
                  "tower"]


def profile_enable(on):
    """False/True = off/every class alone; 2 = gemm_dw only, concurrent on
    its side stream (dcnr_profile_enable)."""
    load().dcnr_profile_enable(int(on))


def profile_collect(with_bytes: bool = False):
    """{class: (total_ms, launches)} since the last collect (synchronises);
    with_bytes: {class: (total_ms, launches, algorithmic_bytes)}."""
    n = len(KERNEL_CLASSES)
    ms = (ctypes.c_double * n)()
    cnt = (ctypes.c_int64 * n)()
    nb = (ctypes.c_double * n)()
    check(load().dcnr_profile_collect_bytes(ctypes.cast(ms, ctypes.c_void_p),
                                            ctypes.cast(cnt, ctypes.c_void_p),
                                            ctypes.cast(nb, ctypes.c_void_p), n), "profile")
    if with_bytes:
        return {k: (ms[i], cnt[i], nb[i]) for i, k in enumerate(KERNEL_CLASSES)}
    return {k: (ms[i], cnt[i]) for i, k in enumerate(KERNEL_CLASSES)}

_lib = None
_lock = threading.Lock()


class LibraryMissing(RuntimeError):
    pass


def load(path: str | None = None):
    """Load (once) and return the bound library.  Raises LibraryMissing."""
    global _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise LibraryMissing(
                f"libdcnr.so not found at {p}: build it with `python -c 'import __graft_entry__ as g; "
                f"g.build()'` (or `make -C <pkg>/csrc`). There is no CPU fallback.")
        lib = ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL)
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        if lib.dcnr_abi_version() != ABI_VERSION:
            raise LibraryMissing("libdcnr ABI version mismatch")
        if path is None:
            _lib = lib
        return lib


def exported_symbols():
    return list(_SIGS.keys())


def check(status: int, what: str = "dcnr"):
    if status == DCNR_OK:
        return
    msg = (load().dcnr_last_error() or b"").decode(errors="replace")
    if status == DCNR_INDEX_OOB:
        raise IndexError(msg or "index out of range in self")
    if status == DCNR_BAD_ARG:
        raise ValueError(f"{what}: {msg}")
    raise RuntimeError(f"{what} failed (status {status}): {msg}")


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def ptr_array(tensors):
    arr = (ctypes.c_void_p * max(1, len(tensors)))()
    for i, t in enumerate(tensors):
        arr[i] = t.data_ptr() if t is not None else None
    return arr
