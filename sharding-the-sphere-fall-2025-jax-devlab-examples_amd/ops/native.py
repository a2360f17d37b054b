"""ctypes binding of the in-tree gfx950 library ``ops/libstsp.so``.

``import torch`` happens first so that the library's ``libamdhip64.so.7`` /
``librccl.so.1`` dependencies resolve to the copies PyTorch already loaded
(same SONAME): one HIP runtime, one device context, torch streams usable.

On a machine with a GPU, a missing or stale library is an error (no silent
fallback); ``require_native()`` raises with the build command.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must precede the library load)

from . import build as _build

_LIB = None
_LOCK = threading.Lock()


class StageDesc(ctypes.Structure):
    _fields_ = [
        ("X", ctypes.c_void_p), ("Q", ctypes.c_void_p), ("acc_in", ctypes.c_void_p),
        ("out", ctypes.c_void_p), ("acc_out", ctypes.c_void_p), ("recv", ctypes.c_void_p),
        ("gmap", ctypes.c_void_p), ("push", ctypes.c_void_p), ("blocks", ctypes.c_void_p),
        ("invA", ctypes.c_void_p), ("ex", ctypes.c_void_p), ("ey", ctypes.c_void_p),
        ("mx", ctypes.c_void_p), ("my", ctypes.c_void_p), ("cgeo", ctypes.c_void_p),
        ("ntile", ctypes.c_int), ("n", ctypes.c_int), ("S", ctypes.c_int), ("mg", ctypes.c_int), ("pw", ctypes.c_int),
        ("nblocks", ctypes.c_int), ("limiter", ctypes.c_int), ("remote", ctypes.c_int),
        ("a0", ctypes.c_double), ("a1", ctypes.c_double), ("a2", ctypes.c_double),
        ("c0", ctypes.c_double), ("c1", ctypes.c_double), ("c2", ctypes.c_double), ("dt", ctypes.c_double),
        ("g", ctypes.c_double), ("omega2", ctypes.c_double),
        ("stamps", ctypes.c_void_p),
        # direct xGMI halo (ops/xgmi.py)
        ("xg", ctypes.c_int), ("ring", ctypes.c_int),
        ("peer_ring", ctypes.c_void_p), ("peer_cnt", ctypes.c_void_p), ("cnt", ctypes.c_void_p),
        ("nprod", ctypes.c_void_p), ("bmask", ctypes.c_void_p), ("epoch", ctypes.c_void_p), ("err", ctypes.c_void_p),
        ("timeout_ticks", ctypes.c_longlong),
        ("pedge", ctypes.c_void_p), ("pe_base", ctypes.c_void_p), ("pe_t", ctypes.c_void_p),
        # streaming stage (march_kernel.hip)
        ("torg", ctypes.c_void_p), ("crec", ctypes.c_void_p), ("lxt", ctypes.c_void_p), ("bpad", ctypes.c_void_p),
        ("Nf", ctypes.c_int), ("frames", ctypes.c_int * 6),
        # carried tile-corner ghosts (parallel/layout.py::corner_sources)
        ("cgmap", ctypes.c_void_p), ("cpush", ctypes.c_void_p),
    ]


class FusedDesc(ctypes.Structure):
    """Mirror of FusedDesc (stsp_kernels.h): one fused SSP-RK3 step."""
    _fields_ = [
        ("Q", ctypes.c_void_p), ("out", ctypes.c_void_p), ("src", ctypes.c_void_p), ("org", ctypes.c_void_p),
        ("len", ctypes.c_void_p), ("nrm", ctypes.c_void_p), ("tane", ctypes.c_void_p), ("crec", ctypes.c_void_p), ("lxt", ctypes.c_void_p), ("gbt", ctypes.c_void_p), ("frames", ctypes.c_int * 6),
        ("code", ctypes.c_void_p),
        ("gtab", ctypes.c_void_p), ("gw", ctypes.c_void_p), ("ctab", ctypes.c_void_p), ("cgf", ctypes.c_void_p),
        ("ccnt", ctypes.c_void_p), ("push", ctypes.c_void_p),
        ("G", ctypes.c_int), ("C", ctypes.c_int),
        ("nblocks", ctypes.c_int), ("n", ctypes.c_int), ("N", ctypes.c_int), ("S", ctypes.c_int),
        ("mg", ctypes.c_int), ("pw", ctypes.c_int), ("B", ctypes.c_int), ("ns", ctypes.c_int),
        ("limiter", ctypes.c_int),
        ("a0", ctypes.c_double * 4), ("a1", ctypes.c_double * 4), ("a2", ctypes.c_double * 4),
        ("dt", ctypes.c_double), ("g", ctypes.c_double), ("omega2", ctypes.c_double),
        ("xg", ctypes.c_int), ("ring", ctypes.c_int), ("recv", ctypes.c_void_p), ("peer_ring", ctypes.c_void_p),
        ("xpush", ctypes.c_void_p), ("K", ctypes.c_int), ("epoch", ctypes.c_void_p), ("err", ctypes.c_void_p),
        ("timeout_ticks", ctypes.c_longlong), ("stamps", ctypes.c_void_p),
        ("local_src", ctypes.c_int), ("links", ctypes.c_int * 6),
        ("nsteps", ctypes.c_int), ("prod", ctypes.c_void_p), ("PM", ctypes.c_int),
        ("cpush", ctypes.c_void_p), ("sched", ctypes.c_void_p), ("nrmf", ctypes.c_void_p),
        ("hx", ctypes.c_void_p), ("pidx", ctypes.c_void_p),
    ]


class March3Desc(ctypes.Structure):
    """Mirror of March3Desc (stsp_kernels.h): the pipelined streaming step."""
    _fields_ = [
        ("q1", ctypes.c_void_p), ("q2", ctypes.c_void_p),
        ("b0", ctypes.c_double * 3), ("b1", ctypes.c_double * 3), ("b2", ctypes.c_double * 3),
        ("D", ctypes.c_int),
    ]


def lib_path() -> str:
    return _build.lib_for(os.environ.get("STSP_VARIANT", ""))


def load(build_if_missing: bool = True):
    """Load (building first if the sources are newer and hipcc exists)."""
    global _LIB
    with _LOCK:
        if _LIB is not None:
            return _LIB
        variant = os.environ.get("STSP_VARIANT", "")
        path = _build.lib_for(variant)
        if build_if_missing and _build.needs_build(variant):
            try:
                _build.build(variant=variant)
            except Exception:
                if not os.path.exists(path):
                    raise
        L = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        vp, ci, cl = ctypes.c_void_p, ctypes.c_int, ctypes.c_long
        L.stsp_stage_launch.argtypes = [ci, ci, ci, ci, ctypes.POINTER(StageDesc), vp]
        L.stsp_stage_launch.restype = ci
        L.stsp_pack_launch.argtypes = [ci, vp, ci, ci, vp, ci, vp, vp]
        L.stsp_pack_launch.restype = ci
        L.stsp_copy_index_launch.argtypes = [ci, vp, vp, vp, vp, ci, ci, cl, cl, vp]
        L.stsp_copy_index_launch.restype = ci
        L.stsp_dpp_probe.argtypes = [vp, vp, vp, vp]
        L.stsp_dpp_probe.restype = ci
        L.stsp_fused_launch.argtypes = [ci, ctypes.POINTER(FusedDesc), vp]
        L.stsp_fused_launch.restype = ci
        L.stsp_march3_launch.argtypes = [ci, ci, ctypes.POINTER(StageDesc), ctypes.POINTER(March3Desc), vp]
        L.stsp_march3_launch.restype = ci
        L.stsp_fused_limits.argtypes = [ctypes.POINTER(ci), ctypes.POINTER(ci)]
        L.stsp_fused_limits.restype = ci
        L.stsp_fused_tagh.argtypes = []
        L.stsp_fused_tagh.restype = ci
        L.stsp_fused_record_words.argtypes = [ci]
        L.stsp_fused_record_words.restype = ci
        L.stsp_fused_prime_launch.argtypes = [ci, vp, ci, vp, vp, ci, vp, ci, ci, vp]
        L.stsp_fused_prime_launch.restype = ci
        _declare_runtime(L)
        _declare_tt(L)
        L.stsp_schedule_spin.argtypes = [ci]
        L.stsp_schedule_spin.restype = ci
        L.stsp_device_flags.argtypes = []
        L.stsp_device_flags.restype = ci
        L.stsp_desc_size.argtypes = [ci]
        L.stsp_desc_size.restype = ci
        for k, cls in ((0, StageDesc), (1, FusedDesc), (3, March3Desc)):
            if L.stsp_desc_size(k) != ctypes.sizeof(cls):
                raise RuntimeError(f"{cls.__name__}: ctypes mirror is {ctypes.sizeof(cls)} bytes, "
                                   f"the library's {L.stsp_desc_size(k)} (stale libstsp.so?)")
        _LIB = L
        return L


def _declare_runtime(L):
    vp, ci, cd = ctypes.c_void_p, ctypes.c_int, ctypes.c_double
    if not hasattr(L, "stsp_rt_create"):
        return
    L.stsp_rt_create.argtypes = [vp]
    L.stsp_rt_create.restype = vp
    L.stsp_rt_destroy.argtypes = [vp]
    L.stsp_rt_destroy.restype = None
    L.stsp_rt_run.argtypes = [vp, ci]
    L.stsp_rt_run.restype = ci
    L.stsp_rt_set_dt.argtypes = [vp, cd]
    L.stsp_rt_set_dt.restype = ci
    L.stsp_rt_last_error.argtypes = [vp]
    L.stsp_rt_last_error.restype = ctypes.c_char_p
    L.stsp_nccl_unique_id.argtypes = [vp]
    L.stsp_nccl_unique_id.restype = ci
    L.stsp_nccl_id_bytes.argtypes = []
    L.stsp_nccl_id_bytes.restype = ci
    L.stsp_rccl_version.argtypes = []
    L.stsp_rccl_version.restype = ci
    L.stsp_rccl_error.argtypes = []
    L.stsp_rccl_error.restype = ctypes.c_char_p
    L.stsp_rccl_path.argtypes = []
    L.stsp_rccl_path.restype = ctypes.c_char_p
    L.stsp_roctx_push.argtypes = [ctypes.c_char_p]
    L.stsp_roctx_push.restype = ci
    L.stsp_roctx_pop.argtypes = []
    L.stsp_roctx_pop.restype = ci


def _declare_tt(L):
    vp, ci, cd = ctypes.c_void_p, ctypes.c_int, ctypes.c_double
    L.stsp_tt_gram_blocks.argtypes = [ci]
    L.stsp_tt_gram_blocks.restype = ci
    L.stsp_tt_gram.argtypes = [ci, vp, ci, vp, ci, ci, ci, ci, vp, ci, vp, ci, cd, vp]
    L.stsp_tt_gram.restype = ci
    L.stsp_tt_mm.argtypes = [ci, vp, ci, vp, ci, vp, ci, ci, ci, ci, cd, cd, vp]
    L.stsp_tt_mm.restype = ci
    L.stsp_tt_chol_inv.argtypes = [ci, vp, ci, ctypes.c_long, vp, vp, ci, ctypes.c_long, ci, ci, cd, vp, vp]
    L.stsp_tt_chol_inv.restype = ci
    L.stsp_tt_expand.argtypes = [ci, vp, ci, vp, ci, ci, ci, cd, cd, cd, cd, cd, ci, vp]
    L.stsp_tt_expand.restype = ci
    L.stsp_tt_dense_diffusion.argtypes = [ci, vp, vp, ci, ci, cd, vp]
    L.stsp_tt_dense_diffusion.restype = ci
    L.stsp_tt_core.argtypes = [ci, vp, cd, ci, vp, ci]
    L.stsp_tt_core.restype = ci
    L.stsp_tt_step_workspace.argtypes = [ci, ci]
    L.stsp_tt_step_workspace.restype = ctypes.c_size_t
    L.stsp_tt_lr_step.argtypes = [ci, vp, ci, vp, ci, ci, ci, cd, cd, ci, cd, ci, vp, vp, vp, vp, ci, vp]
    L.stsp_tt_lr_step.restype = ci
    L.stsp_tt_step_workspace2.argtypes = [ci, ci, ci]
    L.stsp_tt_step_workspace2.restype = ctypes.c_size_t
    L.stsp_tt_lr_step2.argtypes = [ci, vp, ci, vp, ci, ci, ci, ci, cd, cd, ci, cd, ci, vp, vp, vp, vp, ci, vp]
    L.stsp_tt_lr_step2.restype = ci
    L.stsp_tt_set_core.argtypes = [ci]
    L.stsp_tt_set_core.restype = ci
    L.stsp_tt_lr_step3.argtypes = [ci, vp, ci, vp, ci, ci, ci, ci, cd, cd, ci, cd, ci, vp, vp, vp, vp, ci, vp]
    L.stsp_tt_lr_step3.restype = ci
    L.stsp_tt_step_workspace3.argtypes = [ci, ci, ci]
    L.stsp_tt_step_workspace3.restype = ctypes.c_size_t
    L.stsp_tt_recompress_workspace.argtypes = [ci, ci, ci]
    L.stsp_tt_recompress_workspace.restype = ctypes.c_size_t
    L.stsp_tt_recompress.argtypes = [ci, vp, ci, ci, vp, ci, ci, ci, cd, ci, vp, vp, vp, ci, vp, ci, vp]
    L.stsp_tt_recompress.restype = ci
    # persistent factored step (tt_persist.hip)
    L.stsp_tt_persist.argtypes = [vp, ci, vp, ci, ci, ci, ci, ci, cd, cd, ci, cd, ci, vp, vp, vp, vp, ci, vp, vp,
                                  cd, vp]
    L.stsp_tt_persist.restype = ci
    L.stsp_tt_persist_limits.argtypes = [ctypes.POINTER(ci), ctypes.POINTER(ci)]
    L.stsp_tt_persist_limits.restype = ci


def available() -> bool:
    try:
        load()
        return True
    except Exception:
        return False


def require_native():
    try:
        return load()
    except Exception as e:
        raise RuntimeError(
            f"native gfx950 library unavailable ({e}); build it with "
            f"`python -m stsphere.ops.build` (hipcc --offload-arch=gfx950)") from e


def dtype_code(dtype: torch.dtype) -> int:
    if dtype == torch.float64:
        return 1
    if dtype == torch.float32:
        return 0
    raise TypeError(f"unsupported dtype {dtype}")


def ptr(t) -> int:
    return 0 if t is None else int(t.data_ptr())


_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def current_stream_handle(device=None) -> int:
    """hipStream_t of torch's current stream on ``device`` (default: the
    current device).  The raw query skips building a torch.cuda.Stream object
    (microseconds on every launch of a timed region)."""
    if _RAW_STREAM is not None:
        idx = torch.cuda.current_device() if device is None else (
            device.index if isinstance(device, torch.device) and device.index is not None
            else (device if isinstance(device, int) else torch.cuda.current_device()))
        return int(_RAW_STREAM(idx))
    return int(torch.cuda.current_stream(device).cuda_stream)


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed with code {rc}")


def pack(q: torch.Tensor, idx: torch.Tensor, send: torch.Tensor, stream: int = None) -> None:
    L = require_native()
    F, S = q.shape
    assert idx.dtype == torch.int32 and send.numel() >= idx.numel() * F
    rc = L.stsp_pack_launch(dtype_code(q.dtype), ptr(q), S, F, ptr(idx), idx.numel(), ptr(send),
                            current_stream_handle() if stream is None else stream)
    check(rc, "pack")


def copy_index(src: torch.Tensor, sidx: torch.Tensor, dst: torch.Tensor, didx: torch.Tensor, batch: int,
               src_stride: int, dst_stride: int) -> None:
    L = require_native()
    assert sidx.numel() == didx.numel()
    assert sidx.dtype == torch.int32 and didx.dtype == torch.int32
    rc = L.stsp_copy_index_launch(dtype_code(src.dtype), ptr(src), ptr(sidx), ptr(dst), ptr(didx), sidx.numel(),
                                  batch, src_stride, dst_stride, current_stream_handle())
    check(rc, "copy_index")
