"""PyTorch-facing wrappers of the gfx950 low-rank kernels (ops/csrc/tt_kernels.hip).

* ``gram(A, B)``            A^T B for tall-skinny A [N, k], B [N, m] (k, m <= 64), MFMA
* ``tsmm(A, X, out=...)``   A X (+ beta out) for A [N, k], X [k, m], MFMA
* ``expand(X, ...)``        [x0 X + x1 D X, y0 X + y1 D X] with D the 1-D second difference
* ``dense_diffusion(U, c)`` U + c * (5-point Laplacian of U), zero Dirichlet
* ``recompress(A, B, eps)`` A B^T (k <= 64 columns) rounded to rank <= max_rank:
  CholeskyQR3 of both factors + k x k core + two products, ONE native call

All of them run on torch's current stream.  Operands must be CUDA tensors of
one dtype (float64 or float32) whose rows are contiguous (stride(1) == 1); row
strides are passed through, so column slices of a wider matrix work.
These are the "r x r x r multiplies" of the slide-19 TT cost model
(PDF s.19, s.5: TT numerics turn the memory-bound FV update compute-bound).
"""
from __future__ import annotations

import torch

from . import native


def _check(*ts):
    dt = ts[0].dtype
    for t in ts:
        if t.device.type != "cuda":
            raise ValueError("tt_ops need CUDA tensors")
        if t.dtype != dt:
            raise TypeError("operands must share one dtype")
        if t.dim() != 2 or t.stride(1) != 1:
            raise ValueError("operands must be 2-D with contiguous rows")
    return native.dtype_code(dt)


def gram_blocks(N: int) -> int:
    return native.require_native().stsp_tt_gram_blocks(int(N))


def _ceil16(x: int) -> int:
    return (x + 15) // 16 * 16


def gram(A: torch.Tensor, B: torch.Tensor, alpha: float = 1.0, out: torch.Tensor = None,
         work: torch.Tensor = None) -> torch.Tensor:
    """alpha * A^T B  ([k, m]); the reduction over rows runs in a fixed order
    (bitwise reproducible)."""
    L = native.require_native()
    code = _check(A, B)
    N, k = A.shape
    N2, m = B.shape
    if N2 != N or not (1 <= k <= 64 and 1 <= m <= 64):
        raise ValueError(f"gram: shapes {tuple(A.shape)} / {tuple(B.shape)}")
    if out is None:
        out = torch.empty((k, m), dtype=A.dtype, device=A.device)
    _check(out)
    P = L.stsp_tt_gram_blocks(N)
    need = P * _ceil16(k) * _ceil16(m)
    if work is None or work.numel() < need or work.dtype != A.dtype:
        work = torch.empty(need, dtype=A.dtype, device=A.device)
    rc = L.stsp_tt_gram(code, native.ptr(A), A.stride(0), native.ptr(B), B.stride(0), N, k, m, native.ptr(work), P,
                        native.ptr(out), out.stride(0), float(alpha), native.current_stream_handle())
    native.check(rc, "tt_gram")
    return out


def tsmm(A: torch.Tensor, X: torch.Tensor, out: torch.Tensor = None, alpha: float = 1.0,
         beta: float = 0.0) -> torch.Tensor:
    """alpha * A X + beta * out  ([N, m])."""
    L = native.require_native()
    N, k = A.shape
    k2, m = X.shape
    if k2 != k or not (1 <= k <= 64 and 1 <= m <= 64):
        raise ValueError(f"tsmm: shapes {tuple(A.shape)} x {tuple(X.shape)}")
    if out is None:
        if beta != 0.0:
            raise ValueError("beta != 0 needs out")
        out = torch.empty((N, m), dtype=A.dtype, device=A.device)
    code = _check(A, X, out)
    if out.shape != (N, m):
        raise ValueError("tsmm: bad out shape")
    rc = L.stsp_tt_mm(code, native.ptr(A), A.stride(0), native.ptr(X), X.stride(0), native.ptr(out), out.stride(0),
                      N, k, m, float(alpha), float(beta), native.current_stream_handle())
    native.check(rc, "tt_mm")
    return out


def chol_inv(G: torch.Tensor, shift_c: float = 0.0):
    """Batched shifted Cholesky of k x k Gram matrices G [b, k, k] (k <= 64):
    G_i + shift_c trace(G_i) I = R_i^T R_i (shift_c < 0: unshifted unless a
    pivot fails, then shifted by |shift_c|).  Returns (R, R^-1, info) with R
    upper triangular [b, k, k] and info [b] int32 (0, or failing pivot + 1;
    read it only where a host sync happens anyway)."""
    L = native.require_native()
    if G.dim() == 2:
        G = G.unsqueeze(0)
    b, k, k2 = G.shape
    if k != k2 or not 1 <= k <= 64 or G.stride(2) != 1:
        raise ValueError(f"chol_inv: shape {tuple(G.shape)}")
    code = _check(G[0])
    R = torch.empty((b, k, k), dtype=G.dtype, device=G.device)
    Ri = torch.empty_like(R)
    info = torch.empty(b, dtype=torch.int32, device=G.device)
    rc = L.stsp_tt_chol_inv(code, native.ptr(G), G.stride(1), G.stride(0), native.ptr(R), native.ptr(Ri), k, k * k, k, b,
                            float(shift_c), native.ptr(info), native.current_stream_handle())
    native.check(rc, "tt_chol_inv")
    return R, Ri, info


def expand(X: torch.Tensor, x0: float, x1: float, y0: float, y1: float, ih2: float, periodic: bool = False,
           out: torch.Tensor = None) -> torch.Tensor:
    """[N, 2r] = [x0 X + x1 D X, y0 X + y1 D X], (D X)_i = (X_{i-1} - 2 X_i + X_{i+1}) ih2."""
    L = native.require_native()
    N, r = X.shape
    if out is None:
        out = torch.empty((N, 2 * r), dtype=X.dtype, device=X.device)
    code = _check(X, out)
    if out.shape[0] != N or out.shape[1] < 2 * r:
        raise ValueError("expand: bad out shape")
    rc = L.stsp_tt_expand(code, native.ptr(X), X.stride(0), native.ptr(out), out.stride(0), N, r, x0, x1, y0, y1, ih2,
                          int(periodic), native.current_stream_handle())
    native.check(rc, "tt_expand")
    return out


def dense_diffusion(U: torch.Tensor, c: float, out: torch.Tensor = None) -> torch.Tensor:
    """U + c (U_{i-1,j} + U_{i+1,j} + U_{i,j-1} + U_{i,j+1} - 4 U_ij), zero outside."""
    L = native.require_native()
    if not U.is_contiguous():
        raise ValueError("dense_diffusion: U must be contiguous")
    if out is None:
        out = torch.empty_like(U)
    code = _check(U, out)
    N, M = U.shape
    rc = L.stsp_tt_dense_diffusion(code, native.ptr(U), native.ptr(out), N, M, float(c),
                                   native.current_stream_handle())
    native.check(rc, "tt_dense_diffusion")
    return out


class _RecompressBuffers:
    """Device workspace and pinned host buffer of ``recompress``, grown to the
    largest (rows, k) seen and reused (pinning host memory costs milliseconds,
    a recompression tens of microseconds)."""

    def __init__(self):
        self.ws = None
        self.hbuf = None

    def get(self, L, NA: int, NB: int, k: int, dtype, device):
        need = L.stsp_tt_recompress_workspace(NA, NB, k)
        if self.ws is None or self.ws.numel() < need or self.ws.dtype != dtype or self.ws.device != device:
            self.ws = torch.empty(need, dtype=dtype, device=device)
        if self.hbuf is None:
            self.hbuf = torch.empty(8 * 64 * 64 + 8, dtype=torch.float64).pin_memory()
        return self.ws, self.hbuf


_RBUF = _RecompressBuffers()


def recompress(A: torch.Tensor, B: torch.Tensor, eps: float, max_rank: int = None):
    """A [NA, k] B[NB, k]^T -> (A', B') of rank rn <= max_rank with
    ||A B^T - A' B'^T|| <= eps ||A B^T|| (k <= 64; stsp_tt_recompress in
    ops/csrc/tt_kernels.hip): CholeskyQR3 of each factor on the MFMA Gram /
    Cholesky / product kernels, the k x k core on the device (k <= 32; host
    Jacobi above), two MFMA products.  One 4-byte read-back (the rank sizes
    the outputs).  The inputs are not written; the outputs are column slices
    of one [NA + NB, kmax] buffer with contiguous rows."""
    L = native.require_native()
    code = _check(A, B)
    NA, k = A.shape
    NB, k2 = B.shape
    if k2 != k or not 1 <= k <= 64:
        raise ValueError(f"recompress: shapes {tuple(A.shape)} / {tuple(B.shape)}")
    ws, hbuf = _RBUF.get(L, NA, NB, k, A.dtype, A.device)
    rmax = k if not max_rank else min(k, int(max_rank))
    out = torch.empty((NA + NB, rmax), dtype=A.dtype, device=A.device)
    rn = L.stsp_tt_recompress(code, native.ptr(A), A.stride(0), NA, native.ptr(B), B.stride(0), NB, k, float(eps),
                              int(max_rank or 0), native.ptr(ws), native.ptr(hbuf), native.ptr(out), rmax,
                              native.ptr(out[NA:]), rmax, native.current_stream_handle())
    if rn == -22:           # the product is exactly zero: the rank-1 zero field
        z = out[:, :1].zero_()
        return z[:NA], z[NA:]
    if rn <= 0:
        raise RuntimeError(f"stsp_tt_recompress failed ({rn})")
    return out[:NA, :rn], out[NA:, :rn]
