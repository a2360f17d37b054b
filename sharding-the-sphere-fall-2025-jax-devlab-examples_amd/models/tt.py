"""Tensor-Train (TT) numerics (PDF s.3, s.5, s.19).

The reference's research direction: compress N x N panel fields to
O(d N r^2) TT form and run the FV numerics on the compressed representation
(LANL: 124x on Cartesian shallow water, PDF s.3), turning a memory-bound
stencil into matrix-shaped (compute-bound) work (PDF s.5, s.19).

Implemented here (PyTorch; every heavy op is a GEMM / QR / small SVD, which on
MI355X runs on the matrix cores through hipBLASLt / rocSOLVER):

* ``tt_svd``        TT decomposition of a d-way tensor (Oseledets 2011), by
                    relative accuracy or maximal rank
* ``tt_full``       reconstruction;  ``tt_round`` re-compression (QR + SVD)
* ``tt_add``, ``tt_scale``, ``tt_dot``, ``tt_norm``
* ``qtt_reshape`` / ``qtt_unreshape``: quantized TT of a 2^k x 2^k field
* ``LowRankField``  a 2-D field U = A B^T (the d = 2 TT)
* ``LowRankDiffusion``: explicit diffusion  U <- U + dt kappa (D U + U D^T)
                    on a uniform panel, carried out entirely in factored form:
                    factors grow to rank 3r, then QR + SVD truncation back to
                    <= r (rank-adaptive with a tolerance).  ``backend="hip"``
                    runs the step on the gfx950 kernels of ops/tt_ops.py
                    (rank-2r expansion, CholeskyQR3 with MFMA Gram matrices,
                    the shifted-Cholesky kernel and MFMA tall-skinny
                    products; the k x k core SVD on the host)
* ``CubedSphereLowRankDiffusion``: the same factored diffusion on all six
                    panels of the cube, coupled through the cube's halo in
                    factored form (each panel side's ghost strip is gathered as
                    rows of the neighbour's factors, O(N r) instead of the
                    N x N field; orientation from the tile layout's ghost map)
* ``CubedSphereLowRankAdvection``: tracer advection (TC1 cosine bell) on the
                    six panels in factored form with the sphere metric
                    (edge-normal transport, areas), central FV + SSP-RK3,
                    coefficients factored once, Khatri-Rao products
* ``compress_cubed_sphere``: per-panel TT ranks / errors of a [6, N, N] field
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch


# ----------------------------------------------------------------------------
# general d-way TT
# ----------------------------------------------------------------------------

def _trunc_rank(s: torch.Tensor, delta: float, max_rank: Optional[int]) -> int:
    """Smallest rank whose discarded tail has Frobenius norm <= delta."""
    tail = torch.flip(torch.cumsum(torch.flip(s * s, [0]), 0), [0])   # tail[k] = sum_{i>=k} s_i^2
    ok = (tail <= delta * delta).nonzero()
    r = int(ok[0]) if ok.numel() else len(s)
    r = max(1, r)
    if max_rank is not None:
        r = min(r, max_rank)
    return r


def tt_svd(x: torch.Tensor, eps: float = 1e-10, max_rank: Optional[int] = None) -> List[torch.Tensor]:
    """Cores G_k of shape (r_{k-1}, n_k, r_k) with ||x - tt_full(G)|| <= eps ||x||."""
    dims = list(x.shape)
    d = len(dims)
    delta = eps * float(torch.linalg.norm(x)) / math.sqrt(max(d - 1, 1))
    cores = []
    c = x.reshape(dims[0], -1)
    r = 1
    for k in range(d - 1):
        c = c.reshape(r * dims[k], -1)
        u, s, vh = torch.linalg.svd(c, full_matrices=False)
        rk = _trunc_rank(s, delta, max_rank)
        cores.append(u[:, :rk].reshape(r, dims[k], rk))
        c = s[:rk, None] * vh[:rk]
        r = rk
    cores.append(c.reshape(r, dims[-1], 1))
    return cores


def tt_full(cores: Sequence[torch.Tensor]) -> torch.Tensor:
    out = cores[0]
    for g in cores[1:]:
        out = torch.tensordot(out, g, dims=([out.ndim - 1], [0]))
    return out.squeeze(0).squeeze(-1)


def tt_ranks(cores) -> List[int]:
    return [1] + [g.shape[2] for g in cores]


def tt_storage(cores) -> int:
    return sum(g.numel() for g in cores)


def tt_scale(cores, a: float):
    out = [g.clone() for g in cores]
    out[0] = out[0] * a
    return out


def tt_add(a, b):
    """Exact sum (ranks add)."""
    d = len(a)
    out = []
    for k in range(d):
        ga, gb = a[k], b[k]
        if k == 0:
            out.append(torch.cat([ga, gb], dim=2))
        elif k == d - 1:
            out.append(torch.cat([ga, gb], dim=0))
        else:
            ra0, n, ra1 = ga.shape
            rb0, _, rb1 = gb.shape
            z = ga.new_zeros((ra0 + rb0, n, ra1 + rb1))
            z[:ra0, :, :ra1] = ga
            z[ra0:, :, ra1:] = gb
            out.append(z)
    return out


def tt_dot(a, b) -> torch.Tensor:
    """<a, b> without forming the full tensors."""
    v = a[0].new_ones((1, 1))
    for ga, gb in zip(a, b):
        # v[i,j] -> sum over i,j,n of v[i,j] ga[i,n,k] gb[j,n,l]
        t = torch.tensordot(v, ga, dims=([0], [0]))           # (j, n, k)
        v = torch.tensordot(t, gb, dims=([0, 1], [0, 1]))     # (k, l)
    return v.reshape(())


def tt_norm(a) -> float:
    return float(torch.sqrt(torch.clamp(tt_dot(a, a), min=0)))


def tt_round(cores, eps: float = 1e-10, max_rank: Optional[int] = None):
    """Right-to-left QR orthogonalisation, then left-to-right truncated SVD."""
    cores = [g.clone() for g in cores]
    d = len(cores)
    for k in range(d - 1, 0, -1):
        r0, n, r1 = cores[k].shape
        q, rr = torch.linalg.qr(cores[k].reshape(r0, n * r1).T)
        cores[k] = q.T.reshape(-1, n, r1)
        cores[k - 1] = torch.tensordot(cores[k - 1], rr.T, dims=([2], [0]))
    nrm = float(torch.linalg.norm(cores[0]))
    delta = eps * nrm / math.sqrt(max(d - 1, 1))
    for k in range(d - 1):
        r0, n, r1 = cores[k].shape
        u, s, vh = torch.linalg.svd(cores[k].reshape(r0 * n, r1), full_matrices=False)
        rk = _trunc_rank(s, delta, max_rank)
        cores[k] = u[:, :rk].reshape(r0, n, rk)
        cores[k + 1] = torch.tensordot(s[:rk, None] * vh[:rk], cores[k + 1], dims=([1], [0]))
    return cores


def qtt_reshape(f: torch.Tensor) -> torch.Tensor:
    """2^k x 2^k field -> 2 x 4 x ... quantized tensor with interleaved
    (row bit, column bit) pairs, most significant first: a smooth field has low
    QTT ranks."""
    n = f.shape[0]
    k = int(round(math.log2(n)))
    assert f.shape == (n, n) and 2 ** k == n
    t = f.reshape([2] * (2 * k))
    perm = [p for i in range(k) for p in (i, k + i)]
    return t.permute(perm).reshape([4] * k)


def qtt_unreshape(t: torch.Tensor) -> torch.Tensor:
    k = t.ndim
    n = 2 ** k
    x = t.reshape([2] * (2 * k))
    perm = [2 * i for i in range(k)] + [2 * i + 1 for i in range(k)]
    return x.permute(perm).reshape(n, n)


# ----------------------------------------------------------------------------
# d = 2: low-rank panel fields and factored diffusion
# ----------------------------------------------------------------------------

@dataclass
class LowRankField:
    A: torch.Tensor   # [N, r]
    B: torch.Tensor   # [M, r]

    @classmethod
    def from_dense(cls, U: torch.Tensor, eps: float = 1e-10, max_rank: Optional[int] = None) -> "LowRankField":
        """Truncated SVD of a dense field (setup, not a step).  rocSOLVER's
        gesvd gives up on exactly-zero inputs (a field at rest): those are the
        rank-1 zero field, and a device SVD that fails to converge is redone on
        the host in fp64."""
        if not bool(U.any()):
            z = torch.zeros((U.shape[0], 1), dtype=U.dtype, device=U.device)
            return cls(z, torch.zeros((U.shape[1], 1), dtype=U.dtype, device=U.device))
        try:
            u, s, vh = torch.linalg.svd(U, full_matrices=False)
        except RuntimeError:
            Uh = U.detach().to(device="cpu", dtype=torch.float64)
            u, s, vh = (x.to(device=U.device, dtype=U.dtype) for x in torch.linalg.svd(Uh, full_matrices=False))
        r = _trunc_rank(s, eps * float(torch.linalg.norm(U)), max_rank)
        return cls(u[:, :r] * s[:r], vh[:r].T.contiguous())

    @property
    def rank(self) -> int:
        return self.A.shape[1]

    def dense(self) -> torch.Tensor:
        return self.A @ self.B.T

    def storage(self) -> int:
        return self.A.numel() + self.B.numel()


def recompress(A: torch.Tensor, B: torch.Tensor, eps: float, max_rank: Optional[int]) -> LowRankField:
    """A B^T of rank k -> rank <= max_rank with relative accuracy eps:
    two thin QRs (N x k) and one k x k SVD."""
    qa, ra = torch.linalg.qr(A)
    qb, rb = torch.linalg.qr(B)
    u, s, vh = torch.linalg.svd(ra @ rb.T)
    r = _trunc_rank(s, eps * float(torch.linalg.norm(s)), max_rank)
    return LowRankField(qa @ (u[:, :r] * s[:r]), qb @ vh[:r].T)


def cholqr3_shift(N: int, k: int, dtype) -> float:
    """Shift coefficient of shifted CholeskyQR (Fukaya, Kannan, Nakatsukasa,
    Yamamoto, Yanagisawa 2020): s = 11 (N k + k (k + 1)) u trace(G)."""
    return 11.0 * (N * k + k * (k + 1)) * (torch.finfo(dtype).eps / 2)


def cholqr3(X: torch.Tensor, backend: str = "torch"):
    """X [N, k] = Q R by three shifted CholeskyQR passes: Q orthonormal to
    working precision (the Gram/eigen route stops at sqrt(eps)), every pass a
    Gram matrix, a k x k Cholesky and a tall-skinny product.  Pass 1 is
    shifted; passes 2 and 3 shift only where a pivot fails, which keeps the
    factorisation defined for rank-deficient X (the expanded factors repeat
    columns): X = Q R still holds and Q's near-null directions carry no
    weight in a product.  backend "hip": MFMA Gram and
    products (ops/tt_ops.gram / tsmm) and the one-workgroup Cholesky + inverse
    kernel (tt_ops.chol_inv), no host round trip.  Returns (Q, R, info) with
    info a device tensor, nonzero where a pivot failed."""
    N, k = X.shape
    c = cholqr3_shift(N, k, X.dtype)
    Q, R, infos = X, None, []
    for p in range(3):
        # pass 1 always shifted; passes 2 and 3 plain unless a pivot fails
        if backend == "hip":
            from ..ops import tt_ops
            G = tt_ops.gram(Q, Q)
            Rk, Rik, info = tt_ops.chol_inv(G, c if p == 0 else -c)
            Rk = Rk[0]
            Q = tt_ops.tsmm(Q, Rik[0])
        else:
            G = Q.T @ Q
            eye = torch.eye(k, dtype=X.dtype, device=X.device)
            Lc, info = torch.linalg.cholesky_ex(G + (c * torch.trace(G)) * eye if p == 0 else G)
            if p > 0 and int(info) != 0:
                Lc, info = torch.linalg.cholesky_ex(G + (c * torch.trace(G)) * eye)
            Rk = Lc.T
            Q = torch.linalg.solve_triangular(Rk, Q, upper=True, left=False)
            info = info.reshape(1).to(torch.int32)
        R = Rk if R is None else Rk @ R
        infos.append(info)
    return Q, R, torch.cat(infos)


def recompress_many(pairs, eps: float, max_rank: Optional[int], backend: str = "torch") -> List[LowRankField]:
    """Recompress several products A_i B_i^T at once: CholeskyQR3 of every
    factor on the device, the k x k cores R_a R_b^T copied to the host in ONE
    transfer (with the pivot flags), an SVD and truncation per core there, and
    the truncated factors Q_a (U S)_r, Q_b V_r back on the device."""
    qs, cores, infos = [], [], []
    for A, B in pairs:
        qa, ra, ia = cholqr3(A, backend)
        qb, rb, ib = cholqr3(B, backend)
        qs.append((qa, qb))
        cores.append((ra @ rb.T).reshape(-1))
        infos += [ia, ib]
    flat = torch.cat(cores + [torch.cat(infos).to(cores[0].dtype)]).double().cpu()
    nflag = sum(int(i.numel()) for i in infos)
    if bool((flat[flat.numel() - nflag:] != 0).any()):
        raise RuntimeError("CholeskyQR: a shifted Cholesky pivot failed (non-finite factors?)")
    out, o = [], 0
    for (qa, qb), (A, B) in zip(qs, pairs):
        ka, kb = A.shape[1], B.shape[1]
        C = flat[o:o + ka * kb].view(ka, kb).numpy()
        o += ka * kb
        u, sv, vt = np.linalg.svd(C)
        tail = np.cumsum((sv * sv)[::-1])[::-1]
        ok = np.nonzero(tail <= (eps * eps) * max(tail[0], 1e-300))[0]
        r = max(1, int(ok[0]) if ok.size else len(sv))
        if max_rank is not None:
            r = min(r, max_rank)
        Xa = torch.as_tensor(np.ascontiguousarray(u[:, :r] * sv[:r]), dtype=A.dtype, device=A.device)
        Xb = torch.as_tensor(np.ascontiguousarray(vt[:r].T), dtype=B.dtype, device=B.device)
        if backend == "hip":
            from ..ops import tt_ops
            out.append(LowRankField(tt_ops.tsmm(qa, Xa), tt_ops.tsmm(qb, Xb)))
        else:
            out.append(LowRankField(qa @ Xa, qb @ Xb))
    return out


def second_difference(n: int, h: float, bc: str = "dirichlet", dtype=torch.float64, device="cpu") -> torch.Tensor:
    D = torch.zeros((n, n), dtype=dtype, device=device)
    i = torch.arange(n, device=device)
    D[i, i] = -2.0
    D[i[:-1], i[:-1] + 1] = 1.0
    D[i[1:], i[1:] - 1] = 1.0
    if bc == "periodic":
        D[0, n - 1] = 1.0
        D[n - 1, 0] = 1.0
    return D / (h * h)


class LowRankDiffusion:
    """u_t = kappa (u_xx + u_yy) on a uniform N x N panel, forward Euler, in
    factored form U = A B^T:  D U + U D^T = (D A) B^T + A (D B)^T, so
    U + dt kappa lap U = [A, c D A, c A] [B, B, D B]^T  (c = dt kappa), rank 3r,
    recompressed every step."""

    def __init__(self, N: int, L: float = 1.0, kappa: float = 1.0, bc: str = "dirichlet",
                 eps: float = 1e-10, max_rank: Optional[int] = None, dtype=torch.float64, device="cpu",
                 backend: str = "torch", substeps: int = 1, qr: str = "cholqr3n", core: str = "device"):
        self.h = L / (N + 1) if bc == "dirichlet" else L / N
        # hip recompression: "cholqr3n" (default: device CholeskyQR3,
        # machine-precision factors, the whole step in one native call,
        # stsp_tt_lr_step3, 181 -> 115 us with 2 substeps against ~540 us
        # composed in Python, profiles/r3_tt), "cholqr3" (the same composed in
        # Python, recompress_many) or "gram" (the native Gram/eigen step,
        # ~sqrt(eps) accuracy; kept for comparison)
        if qr not in ("cholqr3", "cholqr3n", "gram"):
            raise ValueError(f"unknown qr {qr!r}")
        if core not in ("device", "host"):
            raise ValueError(f"unknown core {core!r}")
        self.qr = qr
        # "cholqr3n": the k x k core (R products, Jacobi SVD, truncation) on the
        # device for k <= 32 (tt_core_kernel; one 4-byte read-back per step)
        # or on the host (six R factors down, the core maps up)
        self.core = core
        self.bc = bc
        self.kappa = kappa
        self.eps = eps
        self.max_rank = max_rank
        self.dt_max = self.h * self.h / (4.0 * kappa)
        if backend not in ("torch", "hip"):
            raise ValueError(f"unknown backend {backend!r}")
        self.backend = backend
        # explicit steps per call; the factors grow exactly (rank x 2 per step)
        # and are recompressed once at the end (the hip step is latency-bound:
        # one host round trip per call, so rounding every second step halves
        # its cost per step; tools/tt_bench.py)
        if substeps < 1:
            raise ValueError("substeps must be >= 1")
        self.substeps = substeps
        # the hip path never forms the N x N operator
        self.D = second_difference(N, self.h, bc, dtype, device) if backend == "torch" else None

    def step(self, U: LowRankField, dt: float) -> LowRankField:
        """``substeps`` explicit steps of size dt, one recompression."""
        if self.backend == "hip" and self.qr == "gram":
            return self._step_hip(U, dt)
        if self.backend == "hip":
            return self._step_hip_cqr(U, dt)
        c = dt * self.kappa
        if self.substeps == 1:
            A = torch.cat([U.A, c * (self.D @ U.A), c * U.A], dim=1)
            B = torch.cat([U.B, U.B, self.D @ U.B], dim=1)
            return recompress(A, B, self.eps, self.max_rank)
        A, B = U.A, U.B
        for _ in range(self.substeps):     # exact rank-doubling form [A, c D A] [B + c D B, B]^T
            A, B = torch.cat([A, c * (self.D @ A)], dim=1), torch.cat([B + c * (self.D @ B), B], dim=1)
        return recompress(A, B, self.eps, self.max_rank)

    def run_persistent(self, U: LowRankField, dt: float, ncalls: int,
                       stamps: Optional[torch.Tensor] = None) -> LowRankField:
        """``ncalls`` factored steps (each ``substeps`` explicit substeps and
        one CholeskyQR3 recompression, the numerics of ``qr="cholqr3n"``) in
        ONE launch of the persistent kernel (ops/csrc/tt_persist.hip): two
        workgroups keep the factors in LDS across the steps and hand the k x k
        core between them on the device.  fp64, N <= 1024, 2^substeps r <= 16,
        N k <= 12288.  The new rank is read once, after the launch.
        ``stamps``: optional int64 [ncalls, 2, 16] device tensor of per-phase
        shader clocks (expand, three QR passes, core hand-offs, product)."""
        from ..ops import native
        L = native.require_native()
        N, r = U.A.shape
        ns = self.substeps
        if U.A.dtype != torch.float64 or U.A.device.type != "cuda":
            raise ValueError("persistent factored step: fp64 CUDA factors")
        A = U.A if U.A.stride(1) == 1 else U.A.contiguous()
        B = U.B if U.B.stride(1) == 1 else U.B.contiguous()
        dev = A.device
        kmax = 16
        out = torch.empty((2, N, kmax), dtype=torch.float64, device=dev)
        key = ("persist", dev)
        if getattr(self, "_pkey", None) != key:
            self._pxch = torch.zeros(512, dtype=torch.float64, device=dev)
            self._pflags = torch.zeros(4, dtype=torch.int32, device=dev)
            self._prn = torch.zeros(1, dtype=torch.int32, device=dev)
            self._pkey = key
        mr = self.max_rank or 0
        rc = L.stsp_tt_persist(native.ptr(A), A.stride(0), native.ptr(B), B.stride(0), N, r, int(ncalls), ns,
                               dt * self.kappa, 1.0 / (self.h * self.h), int(self.bc == "periodic"), self.eps, mr,
                               native.ptr(self._pxch), native.ptr(self._pflags), native.ptr(out[0]),
                               native.ptr(out[1]), kmax, native.ptr(self._prn),
                               native.ptr(stamps) if stamps is not None else None, 2.0,
                               native.current_stream_handle())
        if rc != 0:
            raise RuntimeError(f"stsp_tt_persist failed ({rc})")
        rn = int(self._prn.item())
        if rn <= 0 or int(self._pflags[3].item()) != 0:
            raise RuntimeError(f"persistent factored step failed (rank {rn}, error word {int(self._pflags[3].item())})")
        return LowRankField(out[0, :, :rn], out[1, :, :rn])

    def _step_hip_cqr(self, U: LowRankField, dt: float) -> LowRankField:
        if self.qr == "cholqr3n":
            return self._step_hip_cqr_native(U, dt)
        return self._step_hip_cqr_py(U, dt)

    def _step_hip_cqr_native(self, U: LowRankField, dt: float) -> LowRankField:
        """The rank-doubling form [A, c D A] [B + c D B, B]^T per substep, then
        one CholeskyQR3 recompression, as ONE native call
        (ops/csrc/tt_kernels.hip, stsp_tt_lr_step3: expansion, three passes per
        factor of MFMA Gram / shifted-Cholesky kernel / MFMA product, one host
        round trip for the six k x k R factors, the core SVD on the host, two
        MFMA products).  ``_step_hip_cqr_py`` is the same step composed in
        Python (``recompress_many``)."""
        from ..ops import native
        L = native.require_native()
        N, r = U.A.shape
        ns = self.substeps
        if (r << ns) > 64:
            raise ValueError(f"hip low-rank step: rank {r} x 2^{ns} substeps exceeds the 64-column kernels")
        A = U.A if U.A.stride(1) == 1 else U.A.contiguous()
        B = U.B if U.B.stride(1) == 1 else U.B.contiguous()
        dev, dt_ = A.device, A.dtype
        k = r << ns
        # workspace for the widest step this solver can take (64 columns):
        # allocated once, never per rank change (pinning host memory costs
        # milliseconds, the step ~100 us)
        key = ("cqr", N, ns, dt_, dev)
        if getattr(self, "_wkey3", None) != key:
            rc = 64 >> ns
            self._ws3 = torch.empty(L.stsp_tt_step_workspace3(N, rc, ns), dtype=dt_, device=dev)
            self._hbuf3 = torch.empty(8 * 64 * 64 + 8, dtype=torch.float64).pin_memory()
            self._wkey3 = key
        rmax = k if self.max_rank is None else min(k, self.max_rank)
        out = torch.empty((2, N, rmax), dtype=dt_, device=dev)
        L.stsp_tt_set_core(1 if self.core == "device" else 0)
        rn = L.stsp_tt_lr_step3(native.dtype_code(dt_), native.ptr(A), A.stride(0), native.ptr(B), B.stride(0), N, r,
                                ns, dt * self.kappa, 1.0 / (self.h * self.h), int(self.bc == "periodic"), self.eps,
                                self.max_rank or 0, native.ptr(self._ws3), native.ptr(self._hbuf3),
                                native.ptr(out[0]), native.ptr(out[1]), rmax, native.current_stream_handle())
        if rn <= 0:
            raise RuntimeError(f"stsp_tt_lr_step3 failed ({rn})")
        return LowRankField(out[0, :, :rn], out[1, :, :rn])

    def _step_hip_cqr_py(self, U: LowRankField, dt: float) -> LowRankField:
        from ..ops import tt_ops
        c = dt * self.kappa
        ih2 = 1.0 / (self.h * self.h)
        per = self.bc == "periodic"
        A, B = U.A.contiguous(), U.B.contiguous()
        if (A.shape[1] << self.substeps) > 64:
            raise ValueError(f"hip low-rank step: rank {A.shape[1]} x 2^{self.substeps} substeps exceeds 64 columns")
        for _ in range(self.substeps):
            A, B = tt_ops.expand(A, 1.0, 0.0, 0.0, c, ih2, per), tt_ops.expand(B, 1.0, c, 1.0, 0.0, ih2, per)
        return recompress_many([(A, B)], self.eps, self.max_rank, "hip")[0]

    def _step_hip(self, U: LowRankField, dt: float) -> LowRankField:
        """Same update as ``step`` with the rank-2r form
        U + c (D U + U D^T) = [A, c D A] [B + c D B, B]^T, recompressed through
        the Gram matrices (MFMA) and the 2r x 2r core:
        A^ = Qa Ra with Ra = sqrt(La) Va^T from Ga = Va La Va^T (eigenvalues
        below 1e-13 max dropped: exact rank deficiency is fine), then
        Ra Rb^T = W S Z^T and A' = A^ Va La^-1/2 W_r S_r, B' = B^ Vb Lb^-1/2 Z_r.
        The whole step is one native call (ops/csrc/tt_kernels.hip,
        stsp_tt_lr_step: 6 kernels, one stream sync for the k x k Gram
        matrices, the core on the host in C++ Jacobi).  Going through Gram
        matrices squares the conditioning, so the attainable relative accuracy
        is ~sqrt(machine eps) (1e-8 in fp64)."""
        from ..ops import native
        L = native.require_native()
        N, r = U.A.shape
        ns = self.substeps
        if (r << ns) > 64:
            raise ValueError(f"hip low-rank step: rank {r} x 2^{ns} substeps exceeds the 64-column kernels")
        A = U.A if U.A.stride(1) == 1 else U.A.contiguous()
        B = U.B if U.B.stride(1) == 1 else U.B.contiguous()
        dev, dt_ = A.device, A.dtype
        k = r << ns
        key = (N, ns, dt_, dev)                  # sized for 64 columns, once (see _step_hip_cqr_native)
        if getattr(self, "_wkey", None) != key:
            self._ws = torch.empty(L.stsp_tt_step_workspace2(N, 64 >> ns, ns), dtype=dt_, device=dev)
            self._hbuf = torch.empty(4 * 64 * 64, dtype=torch.float64).pin_memory()
            self._wkey = key
        rmax = k if self.max_rank is None else min(k, self.max_rank)
        out = torch.empty((2, N, rmax), dtype=dt_, device=dev)
        rn = L.stsp_tt_lr_step2(native.dtype_code(dt_), native.ptr(A), A.stride(0), native.ptr(B), B.stride(0), N, r,
                                ns, dt * self.kappa,
                                1.0 / (self.h * self.h), int(self.bc == "periodic"), self.eps,
                                self.max_rank or 0, native.ptr(self._ws), native.ptr(self._hbuf),
                                native.ptr(out[0]), native.ptr(out[1]), rmax, native.current_stream_handle())
        if rn <= 0:
            raise RuntimeError(f"stsp_tt_lr_step failed ({rn})")
        return LowRankField(out[0, :, :rn], out[1, :, :rn])

    def _core(self, G: np.ndarray):
        def half(g):
            lam, V = np.linalg.eigh(0.5 * (g + g.T))
            keep = lam > 1e-13 * max(lam.max(), 1e-300)
            lam, V = lam[keep], V[:, keep]
            sq = np.sqrt(lam)
            return sq[:, None] * V.T, V / sq[None, :]
        Ra, Ia = half(G[0])
        Rb, Ib = half(G[1])
        w, s, zt = np.linalg.svd(Ra @ Rb.T)
        tail = np.cumsum((s * s)[::-1])[::-1]           # tail[j] = sum_{i >= j} s_i^2
        ok = np.nonzero(tail <= (self.eps * self.eps) * tail[0])[0]
        rn = max(1, int(ok[0]) if ok.size else len(s))
        if self.max_rank is not None:
            rn = min(rn, self.max_rank)
        return Ia @ (w[:, :rn] * s[:rn]), Ib @ zt[:rn].T

    def dense_step(self, U: torch.Tensor, dt: float) -> torch.Tensor:
        return U + dt * self.kappa * (self.D @ U + U @ self.D.T)


def _second_diff_rows(X: torch.Tensor) -> torch.Tensor:
    """(D X) with D the unscaled 1-D second difference, zero outside."""
    out = -2.0 * X
    out[1:] += X[:-1]
    out[:-1] += X[1:]
    return out


class CubedSphereLowRankDiffusion:
    """Explicit diffusion on the six panels of the cube in factored form
    (PDF s.3, s.5, s.19: TT numerics on the cubed sphere).

    Each panel field is U_p = A_p B_p^T (rows y, columns x, N x N, uniform
    flat cells of side h), and one forward-Euler step of the five-point
    Laplacian whose ghost cells come from the neighbouring panels (the
    index-space halo of ``TileLayout(N, 1, 1, ng=1)``: the same orientation
    rules as the FV solver's cube-edge exchange, PY:105-163) is

        U_p' = U_p + c (D U_p + U_p D^T) + c (g_W e_0^T + g_E e_{N-1}^T
                                              + e_0 g_S^T + e_{N-1} g_N^T)

    with c = kappa dt / h^2 and g_s the ghost strip of side s, i.e.

        A^ = [A, c D A, c g_W, c g_E, c e_0, c e_{N-1}]
        B^ = [B + c D B, B, e_0, e_{N-1}, g_S, g_N]            (k = 2 r + 4)

    recompressed to rank <= max_rank.  The halo exchange itself is factored:
    ghost j of a strip is the neighbour cell (y, x) = A_q[y] . B_q[x], so a
    side costs O(N r) and no panel is ever expanded.  The coupling is
    symmetric, so the total sum (mass) is conserved up to the truncation.

    backend "torch": thin QRs + a k x k SVD (rocBLAS / rocSOLVER on the GPU);
    backend "hip": CholeskyQR3 of every factor on the device (MFMA Gram and
    tall-skinny products, the shifted-Cholesky kernel), one host transfer of
    the six k x k cores per step (``recompress_many``); qr="gram" keeps the
    earlier Gram/eigen route (native k x k core, ~sqrt(eps) accuracy).  ``dense_step`` is the N x N
    six-panel reference of the same operator."""

    def __init__(self, N: int, kappa: float = 1.0, L: float = 1.0, eps: float = 1e-10,
                 max_rank: Optional[int] = None, dtype=torch.float64, device="cpu", backend: str = "torch",
                 qr: str = "cholqr3"):
        from ..parallel.layout import TileLayout
        if backend not in ("torch", "hip"):
            raise ValueError(f"unknown backend {backend!r}")
        if qr not in ("cholqr3", "gram"):
            raise ValueError(f"unknown qr {qr!r}")
        self.qr = qr
        self.N, self.kappa, self.h = N, kappa, L / N
        self.eps, self.max_rank, self.backend = eps, max_rank, backend
        self.dtype, self.device = dtype, torch.device(device)
        self.dt_max = self.h * self.h / (4.0 * kappa)
        lay = TileLayout(N, 1, 1, ng=1)
        plan = lay.plan(0)
        pw = N + 2
        face_of = [lay.tile_origin(t)[0] for t in plan.tiles]
        src = np.asarray(plan.halo_src, dtype=np.int64)
        dst = np.asarray(plan.halo_dst, dtype=np.int64)
        # ghost slot -> (panel, side, position) and its source cell (panel, y, x)
        self.nbr = [[None] * 4 for _ in range(6)]
        gy = np.full((6, 4, N), -1, np.int64)
        gx = np.full((6, 4, N), -1, np.int64)
        for d, s_ in zip(dst, src):
            tp, r = divmod(int(d), pw * pw)
            py, px = divmod(r, pw)
            py, px = py - 1, px - 1
            tq, r2 = divmod(int(s_), pw * pw)
            qy, qx = divmod(r2, pw)
            qy, qx = qy - 1, qx - 1
            if not (0 <= qy < N and 0 <= qx < N):
                raise RuntimeError("halo source outside the neighbour panel")
            inx, iny = 0 <= px < N, 0 <= py < N
            if iny and px == -1:
                side, pos = 0, py
            elif iny and px == N:
                side, pos = 1, py
            elif inx and py == -1:
                side, pos = 2, px
            elif inx and py == N:
                side, pos = 3, px
            else:
                continue
            p, q = face_of[tp], face_of[tq]
            if self.nbr[p][side] not in (None, q):
                raise RuntimeError("a panel side borders more than one panel")
            self.nbr[p][side] = q
            gy[p, side, pos], gx[p, side, pos] = qy, qx
        if (gy < 0).any():
            raise RuntimeError("incomplete cube halo")
        self.gy = torch.as_tensor(gy, device=self.device)
        self.gx = torch.as_tensor(gx, device=self.device)
        # dense reference: padded [6, N+2, N+2] with the same ghost map, by face
        self._dsrc, self._ddst = [], []
        for d, s_ in zip(dst, src):
            tp, r = divmod(int(d), pw * pw)
            tq, r2 = divmod(int(s_), pw * pw)
            self._ddst.append(face_of[tp] * pw * pw + r)
            self._dsrc.append(face_of[tq] * pw * pw + r2)
        self._ddst = torch.as_tensor(self._ddst, device=self.device)
        self._dsrc = torch.as_tensor(self._dsrc, device=self.device)
        e = torch.zeros((N, 2), dtype=dtype, device=self.device)
        e[0, 0] = 1.0
        e[N - 1, 1] = 1.0
        self._e = e
        self.stats = {"host_syncs": 0}

    def ghosts(self, F: Sequence[LowRankField], p: int) -> torch.Tensor:
        """[4, N] ghost strips (W, E, S, N) of panel p, gathered in factored form."""
        out = []
        for side in range(4):
            q = self.nbr[p][side]
            out.append((F[q].A[self.gy[p, side]] * F[q].B[self.gx[p, side]]).sum(1))
        return torch.stack(out)

    def expanded(self, F: Sequence[LowRankField], dt: float):
        """Per panel (A^, B^) of the step (k = 2 r + 4 columns), from the old fields."""
        c = dt * self.kappa / (self.h * self.h)
        out = []
        for p in range(6):
            A, B = F[p].A, F[p].B
            g = self.ghosts(F, p)
            Ah = torch.cat([A, c * _second_diff_rows(A), c * g[0:2].T, c * self._e], dim=1)
            Bh = torch.cat([B + c * _second_diff_rows(B), B, self._e, g[2:4].T], dim=1)
            out.append((Ah.contiguous(), Bh.contiguous()))
        return out

    def step(self, F: Sequence[LowRankField], dt: float) -> List[LowRankField]:
        ex = self.expanded(F, dt)
        if self.backend == "torch":
            return [recompress(Ah, Bh, self.eps, self.max_rank) for Ah, Bh in ex]
        if self.qr == "cholqr3":
            self.stats["host_syncs"] += 1
            return recompress_many(ex, self.eps, self.max_rank, "hip")
        return self._recompress_hip(ex)

    def _recompress_hip(self, ex) -> List[LowRankField]:
        """Gram route on the gfx950 kernels: 12 MFMA Gram matrices, one copy to
        the host, six native k x k cores, 12 MFMA tall-skinny products."""
        import ctypes
        from ..ops import native, tt_ops
        L = native.require_native()
        ks = [Ah.shape[1] for Ah, _ in ex]          # 2 r_p + 4: the panels' ranks differ
        if max(ks) > 64:
            raise ValueError(f"hip cube step supports rank <= 30 (k = {max(ks)})")
        Gs = []
        for (Ah, Bh), k in zip(ex, ks):
            G = torch.empty((2, k, k), dtype=Ah.dtype, device=Ah.device)
            tt_ops.gram(Ah, Ah, out=G[0])
            tt_ops.gram(Bh, Bh, out=G[1])
            Gs.append(G.reshape(-1))
        Gh = torch.cat(Gs).double().cpu()           # the one host round trip of the step
        self.stats["host_syncs"] += 1
        Xs, ranks, o = [], [], 0
        for k in ks:
            g = Gh[o:o + 2 * k * k].contiguous()
            o += 2 * k * k
            X = torch.zeros((k, 2 * k), dtype=torch.float64)
            rn = L.stsp_tt_core(k, ctypes.c_void_p(g.data_ptr()), float(self.eps), int(self.max_rank or 0),
                                ctypes.c_void_p(X.data_ptr()), 2 * k)
            if rn <= 0:
                raise RuntimeError(f"stsp_tt_core failed ({rn})")
            Xs.append(X)
            ranks.append(rn)
        Xd = torch.cat([X.reshape(-1) for X in Xs]).to(device=ex[0][0].device, dtype=ex[0][0].dtype)
        out, o = [], 0
        for (Ah, Bh), k, rn in zip(ex, ks, ranks):
            X = Xd[o:o + 2 * k * k].view(k, 2 * k)
            o += 2 * k * k
            A2 = tt_ops.tsmm(Ah, X[:, :rn].contiguous())
            B2 = tt_ops.tsmm(Bh, X[:, rn:2 * rn].contiguous())
            out.append(LowRankField(A2, B2))
        return out

    # ---- dense reference / conversions ---------------------------------------
    def to_factored(self, U6: torch.Tensor) -> List[LowRankField]:
        return [LowRankField.from_dense(U6[p].to(self.dtype), self.eps, self.max_rank) for p in range(6)]

    @staticmethod
    def to_dense(F: Sequence[LowRankField]) -> torch.Tensor:
        return torch.stack([f.dense() for f in F])

    def dense_step(self, U6: torch.Tensor, dt: float) -> torch.Tensor:
        N = self.N
        c = dt * self.kappa / (self.h * self.h)
        P = torch.zeros((6, N + 2, N + 2), dtype=U6.dtype, device=U6.device)
        P[:, 1:-1, 1:-1] = U6
        flat = P.reshape(-1)
        flat[self._ddst] = flat[self._dsrc]
        lap = (P[:, :-2, 1:-1] + P[:, 2:, 1:-1]) + (P[:, 1:-1, :-2] + P[:, 1:-1, 2:]) - 4.0 * U6
        return U6 + c * lap


def _setup_svd(M: torch.Tensor):
    """Thin SVD for setup (coefficient factors): device matrices go through
    the host LAPACK in fp64 and the factors come back to M's device.
    rocSOLVER's device SVD takes seconds per 1024^2 panel and left ~1e-9
    relative errors in small factors (profiles/r6_tt/README.md)."""
    if M.device.type == "cuda":
        u, s, vh = torch.linalg.svd(M.detach().to(device="cpu", dtype=torch.float64), full_matrices=False)
        return (x.to(device=M.device, dtype=M.dtype) for x in (u, s, vh))
    return torch.linalg.svd(M, full_matrices=False)


def lowrank_coefficients(M: torch.Tensor, eps: float):
    """Factor a fixed coefficient field M [n, m] as C D^T to relative accuracy eps."""
    u, s, vh = _setup_svd(M)
    r = _trunc_rank(s, eps * float(torch.linalg.norm(s)), None)
    return (u[:, :r] * s[:r]).contiguous(), vh[:r].T.contiguous()


def hadamard(C: torch.Tensor, D: torch.Tensor, A: torch.Tensor, B: torch.Tensor):
    """(C D^T) o (A B^T) = (C * A)(D * B)^T with row-wise Khatri-Rao factors
    (rank rc ra): a variable coefficient times a factored field."""
    n, m = C.shape[0], D.shape[0]
    return ((C[:, :, None] * A[:, None, :]).reshape(n, -1), (D[:, :, None] * B[:, None, :]).reshape(m, -1))


def _face_avg(X: torch.Tensor) -> torch.Tensor:
    """[n, r] cell factor -> [n+1, r] face average 0.5 (X[i-1] + X[i]), zero outside."""
    out = torch.zeros((X.shape[0] + 1, X.shape[1]), dtype=X.dtype, device=X.device)
    out[:-1] += 0.5 * X
    out[1:] += 0.5 * X
    return out


def _face_diff(X: torch.Tensor) -> torch.Tensor:
    """[n+1, r] face factor -> [n, r] difference X[i+1] - X[i]."""
    return X[1:] - X[:-1]


class CubedSphereLowRankAdvection:
    """Tracer advection dq/dt + div(q v) = 0 on the six panels of the cubed
    sphere, carried entirely in factored form U_p = A_p B_p^T (PDF s.13 / s.18
    workload, TT numerics of PDF s.3, s.19; round-2 verdict item 7).

    Finite volumes with the true sphere metric, as the FV solver
    (models/advection.py): edge-normal transport U = (v . m) L at every edge
    midpoint, cell areas A, central edge values and SSP-RK3,

        dq/dt = -(1/A) [ Fx_{i+1/2} - Fx_{i-1/2} + Fy_{j+1/2} - Fy_{j-1/2} ],
        Fx = Ux (q_{i-1} + q_i) / 2.

    The scheme is linear in q, so every operation stays factored: the metric
    coefficients Ux, Uy, 1/A are factored once (``coef_eps``), a coefficient
    times a field is a Khatri-Rao product of factors, the face average and
    difference act on the factors' rows, and the cube coupling is the ghost
    strips of the neighbour panels gathered in factored form (O(N r) each,
    orientation from the FV layout's index-space halo, as
    ``CubedSphereLowRankDiffusion``), added as rank-1 terms.  Ranks are
    truncated to ``eps`` after every product (``recompress``: thin QRs + a
    k x k SVD).  The flux through a panel edge is computed identically on both
    sides (same edge, same ghost pairs), so mass is conserved up to the
    truncation.  ``dense_step`` is the N x N six-panel reference of the same
    operator; tests/test_tt_and_models.py compares both, and the factored TC1
    run with the FV solver's."""

    def __init__(self, N: int, alpha: float = 0.0, eps: float = 1e-10, max_rank: Optional[int] = None,
                 coef_eps: float = 1e-13, u0: Optional[float] = None, dtype=torch.float64, device="cpu"):
        from .geometry import CubedSphereGrid
        from . import initial_conditions as ic
        self.N, self.eps, self.max_rank = N, eps, max_rank
        self.dtype, self.device = dtype, torch.device(device)
        grid = CubedSphereGrid(N)
        self.grid = grid
        self.u0 = u0 if u0 is not None else 2.0 * math.pi * grid.radius / (12.0 * 86400.0)
        self.alpha = alpha
        wind = lambda p: ic.solid_body_wind(p, self.u0, alpha, grid.radius)
        ux = np.sum(wind(grid.x_edge_midpoints()) * grid.x_edge_normals()[:, None, :, :], -1) * grid.x_edge_lengths()
        uy = np.sum(wind(grid.y_edge_midpoints()) * grid.y_edge_normals()[:, :, None, :], -1) * grid.y_edge_lengths()
        t = lambda a: torch.as_tensor(np.ascontiguousarray(a), dtype=dtype, device=self.device)
        self.Ux, self.Uy, self.invA = t(ux), t(uy), t(1.0 / grid.areas())     # dense copies (reference)
        self.cx = [lowrank_coefficients(self.Ux[p], coef_eps) for p in range(6)]
        self.cy = [lowrank_coefficients(self.Uy[p], coef_eps) for p in range(6)]
        self.ca = [lowrank_coefficients(self.invA[p], coef_eps) for p in range(6)]
        self.halo = CubedSphereLowRankDiffusion(N, dtype=dtype, device=device)
        e = torch.zeros((N + 1, 2), dtype=dtype, device=self.device)
        e[0, 0] = 1.0
        e[N, 1] = 1.0
        self._e = e
        self.dt_max = 0.9 * grid.min_spacing() / (2.0 * self.u0)

    def coefficient_ranks(self) -> dict:
        return {"Ux": [c.shape[1] for c, _ in self.cx], "Uy": [c.shape[1] for c, _ in self.cy],
                "invA": [c.shape[1] for c, _ in self.ca]}

    def _trunc(self, A, B) -> LowRankField:
        return recompress(A, B, self.eps, self.max_rank)

    def rhs(self, F: Sequence[LowRankField]) -> List[LowRankField]:
        out = []
        for p in range(6):
            A, B = F[p].A, F[p].B
            g = self.halo.ghosts(F, p)                                    # [4, N]: W, E, S, N strips
            # x faces (rows j, faces i): A avg(B)^T + 0.5 g_W e_0^T + 0.5 g_E e_N^T
            Ax = torch.cat([A, 0.5 * g[0:2].T], 1)
            Bx = torch.cat([_face_avg(B), self._e], 1)
            fx = self._trunc(*hadamard(*self.cx[p], Ax, Bx))
            # y faces (faces j, columns i): avg(A) B^T + 0.5 e_0 g_S^T + 0.5 e_N g_N^T
            Ay = torch.cat([_face_avg(A), self._e], 1)
            By = torch.cat([B, 0.5 * g[2:4].T], 1)
            fy = self._trunc(*hadamard(*self.cy[p], Ay, By))
            div = self._trunc(torch.cat([fx.A, _face_diff(fy.A)], 1), torch.cat([_face_diff(fx.B), fy.B], 1))
            Ca, Da = self.ca[p]
            La, Lb = hadamard(Ca, Da, div.A, div.B)
            out.append(self._trunc(-La, Lb))
        return out

    def _axpy(self, a: float, X: Sequence[LowRankField], b: float, Y: Sequence[LowRankField]) -> List[LowRankField]:
        return [self._trunc(torch.cat([a * x.A, b * y.A], 1), torch.cat([x.B, y.B], 1)) for x, y in zip(X, Y)]

    def step(self, F: Sequence[LowRankField], dt: float) -> List[LowRankField]:
        """One SSP-RK3 step."""
        L0 = self.rhs(F)
        U1 = self._axpy(1.0, F, dt, L0)
        L1 = self.rhs(U1)
        U2 = self._axpy(0.75, F, 0.25, self._axpy(1.0, U1, dt, L1))
        L2 = self.rhs(U2)
        return self._axpy(1.0 / 3.0, F, 2.0 / 3.0, self._axpy(1.0, U2, dt, L2))

    # ---- dense reference of the same operator --------------------------------
    def dense_rhs(self, U6: torch.Tensor) -> torch.Tensor:
        N = self.N
        P = torch.zeros((6, N + 2, N + 2), dtype=U6.dtype, device=U6.device)
        P[:, 1:-1, 1:-1] = U6
        flat = P.reshape(-1)
        flat[self.halo._ddst] = flat[self.halo._dsrc]
        qx = 0.5 * (P[:, 1:-1, :-1] + P[:, 1:-1, 1:])                   # [6, N, N+1]
        qy = 0.5 * (P[:, :-1, 1:-1] + P[:, 1:, 1:-1])                   # [6, N+1, N]
        fx, fy = self.Ux * qx, self.Uy * qy
        return -((fx[:, :, 1:] - fx[:, :, :-1]) + (fy[:, 1:] - fy[:, :-1])) * self.invA

    def dense_step(self, U6: torch.Tensor, dt: float) -> torch.Tensor:
        U1 = U6 + dt * self.dense_rhs(U6)
        U2 = 0.75 * U6 + 0.25 * (U1 + dt * self.dense_rhs(U1))
        return U6 / 3.0 + (2.0 / 3.0) * (U2 + dt * self.dense_rhs(U2))

    def mass(self, U6: torch.Tensor) -> float:
        return float((U6 / self.invA).sum())

    def to_factored(self, U6: torch.Tensor) -> List[LowRankField]:
        return [LowRankField.from_dense(U6[p].to(self.dtype), self.eps, self.max_rank) for p in range(6)]

    @staticmethod
    def to_dense(F: Sequence[LowRankField]) -> torch.Tensor:
        return torch.stack([f.dense() for f in F])


# columns per native rounding call of the six-panel SWE's "hip" backend: the
# device core (tt_core_kernel) takes k <= 32; wider cores go through the host
# Jacobi SVD (~1.7 ms per call at k = 64 measured at N = 256,
# profiles/r6_tt/README.md)
ROUND_CAP = 32


class CubedSphereLowRankShallowWater:
    """Linearised rotating shallow water on the six panels of the cubed
    sphere, carried entirely in factored form U_p = A_p B_p^T: the six-panel
    counterpart of ``LowRankShallowWater`` (the Cartesian 2-D SWEs of the TT
    speed-up the slides cite, PDF s.3) on the reference's own grid (PDF s.4,
    s.19).

    State per panel: the height perturbation h and the velocity as Cartesian
    components (vx, vy, vz), exchanged across panel edges as three scalars, as
    the reference exchanges winds ("Cartesian Velocity Exchange", PDF s.18).
    About a resting layer of depth H:

        h_t = -H div v,    v_t = -g P grad h - f r x v,    f = 2 Omega z,

    finite volumes with the true sphere metric (models/swe.py's geometry):
    central face values, edge lengths L and unit normals m (per grid line),
    exact cell areas A, the Gauss gradient minus its curvature sum
    S = sum L m (so a constant h has no gradient), P = I - r r^T the tangent
    projection at the cell centre r, SSP-RK3.  The operator is linear, so
    every product stays factored: the metric coefficients (L m_c per face,
    S_c, 1/A, r_c, f r_c) are factored once (``coef_eps``), a coefficient
    times a field is a Khatri-Rao product of factors, face averages and
    differences act on the factors' rows, and the cube coupling is the ghost
    strips gathered from the neighbour panels' factors (O(N r) per side;
    ``CubedSphereLowRankDiffusion.ghosts``), added as rank-1 terms.  Ranks are
    truncated to ``eps`` after every product.  A face between two panels sees
    the same two cells from both sides, so the total mass sum(A h) is
    conserved to round-off and truncation.  ``dense_step`` is the N x N
    six-panel reference of the same discrete operator
    (tests/test_tt_and_models.py: factored vs dense to 1e-10).

    ``backend``: "torch" rounds every product with Householder QR + SVD
    (``recompress``); "hip" (CUDA tensors) rounds every product of at most 64
    columns (and no more columns than rows) in ONE native call,
    ``ops/tt_ops.recompress`` = stsp_tt_recompress: CholeskyQR3 of both
    factors on the MFMA Gram / Cholesky / product kernels, the k x k core on
    the device, one 4-byte read-back.  Wider products (a coefficient of rank
    rc times a field of rank rf has rc rf columns) are rounded chunk by chunk
    through the same call (``_round_native``); only a product whose rank
    fills min(32, N / 2) columns stays on the library QR (rocSOLVER) and SVD.
    ``stats`` counts native calls and library roundings
    (tests/test_tt_kernels.py, tools/tt_sphere_bench.py)."""

    FIELDS = ("h", "vx", "vy", "vz")

    def __init__(self, N: int, H: float = 1000.0, g: float = 9.80616, omega: float = 7.292e-5,
                 eps: float = 1e-13, max_rank: Optional[int] = None, coef_eps: float = 1e-15,
                 dtype=torch.float64, device="cpu", backend: str = "torch"):
        from .geometry import CubedSphereGrid
        if backend not in ("torch", "hip"):
            raise ValueError(f"backend must be 'torch' or 'hip', got {backend!r}")
        if backend == "hip" and torch.device(device).type != "cuda":
            raise ValueError("backend 'hip' needs a CUDA device")
        self.backend = backend
        self.N, self.H, self.g, self.omega = N, H, g, omega
        self.eps, self.max_rank = eps, max_rank
        self.dtype, self.device = dtype, torch.device(device)
        grid = CubedSphereGrid(N)
        self.grid = grid
        lx, ly = grid.x_edge_lengths(), grid.y_edge_lengths()          # [6, N, N+1], [6, N+1, N]
        mx, my = grid.x_edge_normals(), grid.y_edge_normals()          # [6, N+1, 3] per grid line
        area = grid.areas()
        r = grid.centers()                                               # [6, N, N, 3]
        cx = lx[..., None] * mx[:, None, :, :]                           # [6, N, N+1, 3]
        cy = ly[..., None] * my[:, :, None, :]                           # [6, N+1, N, 3]
        S = (cx[:, :, 1:] - cx[:, :, :-1]) + (cy[:, 1:] - cy[:, :-1])   # [6, N, N, 3] curvature sum
        f = 2.0 * omega * r[..., 2]
        t = lambda a: torch.as_tensor(np.ascontiguousarray(a), dtype=dtype, device=self.device)
        # dense copies (reference operator)
        self.Cx, self.Cy, self.S = t(cx), t(cy), t(S)
        self.invA, self.r, self.fr = t(1.0 / area), t(r), t(f[..., None] * r)
        fac = lambda M: lowrank_coefficients(M, coef_eps)
        self.kcx = [[fac(self.Cx[p, ..., c]) for c in range(3)] for p in range(6)]
        self.kcy = [[fac(self.Cy[p, ..., c]) for c in range(3)] for p in range(6)]
        self.kS = [[fac(self.S[p, ..., c]) for c in range(3)] for p in range(6)]
        self.kA = [fac(self.invA[p]) for p in range(6)]
        self.kr = [[fac(self.r[p, ..., c]) for c in range(3)] for p in range(6)]
        self.kfr = [[fac(self.fr[p, ..., c]) for c in range(3)] for p in range(6)]
        self.halo = CubedSphereLowRankDiffusion(N, dtype=dtype, device=device)
        e = torch.zeros((N + 1, 2), dtype=dtype, device=self.device)
        e[0, 0] = 1.0
        e[N, 1] = 1.0
        self._e = e
        c = math.sqrt(g * H)
        self.dt_max = 0.5 * grid.min_spacing() / (c + 1e-300)
        self.stats = {"recompressions": 0, "max_k": 0, "native": 0, "library": 0}

    def coefficient_ranks(self) -> dict:
        rk = lambda L: max(int(C.shape[1]) for C, _ in L)
        return {"L m": max(rk(self.kcx[p]) for p in range(6)), "S": max(rk(self.kS[p]) for p in range(6)),
                "1/A": max(int(C.shape[1]) for C, _ in self.kA), "r": max(rk(self.kr[p]) for p in range(6)),
                "f r": max(rk(self.kfr[p]) for p in range(6))}

    # ---- factored operator ----------------------------------------------------
    def _trunc(self, A, B) -> LowRankField:
        self.stats["recompressions"] += 1
        k = int(A.shape[1])
        self.stats["max_k"] = max(self.stats["max_k"], k)
        if self.backend == "hip":
            out = self._round_native(A, B)
            if out is not None:
                return out
            self.stats["library"] += 1
            return self._round_library(A, B)
        self.stats["library"] += 1
        return recompress(A, B, self.eps, self.max_rank)

    def _round_library(self, A, B) -> LowRankField:
        """The hip backend's rounding of a product too wide for the native
        call: Householder QR of both factors on the device (rocSOLVER geqrf),
        the core's SVD on the host in fp64 (LAPACK).  The device SVD of the
        core (rocSOLVER's Jacobi-based gesvd path) left relative errors up to
        4e-9 per rounding where this route and the native call stay near
        1e-12 (profiles/r6_tt/README.md)."""
        qa, ra = torch.linalg.qr(A)
        qb, rb = torch.linalg.qr(B)
        C = (ra @ rb.T).to(device="cpu", dtype=torch.float64).numpy()
        u, sv, vt = np.linalg.svd(C)
        tail = np.cumsum((sv * sv)[::-1])[::-1]
        ok = np.nonzero(tail <= (self.eps * self.eps) * max(tail[0], 1e-300))[0]
        r = max(1, int(ok[0]) if ok.size else len(sv))
        if self.max_rank is not None:
            r = min(r, self.max_rank)
        Xa = torch.as_tensor(np.ascontiguousarray(u[:, :r] * sv[:r]), dtype=A.dtype, device=A.device)
        Xb = torch.as_tensor(np.ascontiguousarray(vt[:r].T), dtype=B.dtype, device=B.device)
        return LowRankField(qa @ Xa, qb @ Xb)

    def _round_native(self, A, B, cap: Optional[int] = None) -> Optional[LowRankField]:
        """Round A B^T with native calls of at most cap = min(ROUND_CAP,
        rows / 2) columns (the k x k core runs on the device up to 32 columns;
        a factor at least twice as tall as wide keeps CholeskyQR well posed):
        the first cap columns, then the running result concatenated
        with the next cap - rank columns, and so on (A B^T is the sum of its
        column chunks' products; each rounding is relative to its partial sum,
        max_rank applies to the last).  A Khatri-Rao product of rc rf columns
        thus costs ~rc (r + rf)^2 N instead of (rc rf)^2 N.  None (library path)
        when the running rank fills the cap."""
        from ..ops import tt_ops
        k = int(A.shape[1])
        if cap is None:
            cap = min(ROUND_CAP, int(A.shape[0]) // 2, int(B.shape[0]) // 2)
        if k <= cap:
            self.stats["native"] += 1
            return LowRankField(*tt_ops.recompress(A, B, self.eps, self.max_rank))
        a, b = tt_ops.recompress(A[:, :cap], B[:, :cap], self.eps)
        calls, o = 1, cap
        while o < k:
            c = cap - int(a.shape[1])
            if c < 1:
                return None
            last = o + c >= k
            a, b = tt_ops.recompress(torch.cat([a, A[:, o:o + c]], 1), torch.cat([b, B[:, o:o + c]], 1), self.eps,
                                     self.max_rank if last else None)
            calls, o = calls + 1, o + c
        self.stats["native"] += calls
        return LowRankField(a, b)

    def _avg_x(self, X: LowRankField, g: torch.Tensor):
        """Face values of x-faces [N, N+1] with the W / E ghost strips."""
        return (torch.cat([X.A, 0.5 * g[0:2].T], 1), torch.cat([_face_avg(X.B), self._e], 1))

    def _avg_y(self, X: LowRankField, g: torch.Tensor):
        return (torch.cat([_face_avg(X.A), self._e], 1), torch.cat([X.B, 0.5 * g[2:4].T], 1))

    def _div(self, kx, ky, ax, ay) -> LowRankField:
        """sum_c  diff_x (Cx_c avg_x(X_c)) + diff_y (Cy_c avg_y(X_c)) over the
        given (coefficient, face-value) pairs, then times 1/A."""
        As, Bs = [], []
        for (Cc, Dc), (A, B) in zip(kx, ax):
            fx = self._trunc(*hadamard(Cc, Dc, A, B))
            As.append(fx.A)
            Bs.append(_face_diff(fx.B))
        for (Cc, Dc), (A, B) in zip(ky, ay):
            fy = self._trunc(*hadamard(Cc, Dc, A, B))
            As.append(_face_diff(fy.A))
            Bs.append(fy.B)
        return self._trunc(torch.cat(As, 1), torch.cat(Bs, 1))

    def _times(self, k, X: LowRankField) -> LowRankField:
        return self._trunc(*hadamard(k[0], k[1], X.A, X.B))

    def rhs(self, F: Sequence[Sequence[LowRankField]]) -> List[List[LowRankField]]:
        """F[q][p]: field q (h, vx, vy, vz) of panel p -> the same for d/dt."""
        out = [[None] * 6 for _ in range(4)]
        for p in range(6):
            gh = [self.halo.ghosts(F[q], p) for q in range(4)]           # [4, N] strips per field
            # h_t = -H (1/A) div v
            div = self._div(self.kcx[p], self.kcy[p], [self._avg_x(F[1 + c][p], gh[1 + c]) for c in range(3)],
                            [self._avg_y(F[1 + c][p], gh[1 + c]) for c in range(3)])
            dh = self._times(self.kA[p], div)
            out[0][p] = LowRankField(-self.H * dh.A, dh.B)
            # Gauss gradient G_c = (1/A) (sum_faces h L m_c - S_c h)
            hx, hy = self._avg_x(F[0][p], gh[0]), self._avg_y(F[0][p], gh[0])
            G = []
            for c in range(3):
                d = self._div([self.kcx[p][c]], [self.kcy[p][c]], [hx], [hy])
                sh = self._times(self.kS[p][c], F[0][p])
                G.append(self._times(self.kA[p], self._trunc(torch.cat([d.A, -sh.A], 1), torch.cat([d.B, sh.B], 1))))
            rG = [self._times(self.kr[p][c], G[c]) for c in range(3)]
            rGs = self._trunc(torch.cat([x.A for x in rG], 1), torch.cat([x.B for x in rG], 1))
            v = [F[1 + c][p] for c in range(3)]
            for c in range(3):
                # -g (G_c - r_c (r . G)) - (f r x v)_c
                a_, b_ = (c + 1) % 3, (c + 2) % 3
                rc = self._times(self.kr[p][c], rGs)
                t1 = self._times(self.kfr[p][a_], v[b_])
                t2 = self._times(self.kfr[p][b_], v[a_])
                out[1 + c][p] = self._trunc(torch.cat([-self.g * G[c].A, self.g * rc.A, -t1.A, t2.A], 1),
                                            torch.cat([G[c].B, rc.B, t1.B, t2.B], 1))
        return out

    def _axpy(self, a: float, X, b: float, Y):
        return [[self._trunc(torch.cat([a * x.A, b * y.A], 1), torch.cat([x.B, y.B], 1)) for x, y in zip(Xq, Yq)]
                for Xq, Yq in zip(X, Y)]

    def step(self, F, dt: float):
        """One SSP-RK3 step of the four factored fields."""
        U1 = self._axpy(1.0, F, dt, self.rhs(F))
        U2 = self._axpy(0.75, F, 0.25, self._axpy(1.0, U1, dt, self.rhs(U1)))
        return self._axpy(1.0 / 3.0, F, 2.0 / 3.0, self._axpy(1.0, U2, dt, self.rhs(U2)))

    # ---- dense reference of the same operator --------------------------------
    def _pad(self, U6: torch.Tensor) -> torch.Tensor:
        N = self.N
        P = torch.zeros((6, N + 2, N + 2), dtype=U6.dtype, device=U6.device)
        P[:, 1:-1, 1:-1] = U6
        flat = P.reshape(-1)
        flat[self.halo._ddst] = flat[self.halo._dsrc]
        return P

    def dense_rhs(self, W: torch.Tensor) -> torch.Tensor:
        """W [4, 6, N, N] = (h, vx, vy, vz)."""
        Ps = [self._pad(W[q]) for q in range(4)]
        avx = lambda P: 0.5 * (P[:, 1:-1, :-1] + P[:, 1:-1, 1:])         # [6, N, N+1]
        avy = lambda P: 0.5 * (P[:, :-1, 1:-1] + P[:, 1:, 1:-1])         # [6, N+1, N]
        dvg = lambda fx, fy: (fx[:, :, 1:] - fx[:, :, :-1]) + (fy[:, 1:] - fy[:, :-1])
        div = sum(dvg(self.Cx[..., c] * avx(Ps[1 + c]), self.Cy[..., c] * avy(Ps[1 + c])) for c in range(3))
        dh = -self.H * self.invA * div
        h = W[0]
        G = torch.stack([self.invA * (dvg(self.Cx[..., c] * avx(Ps[0]), self.Cy[..., c] * avy(Ps[0]))
                                      - self.S[..., c] * h) for c in range(3)])
        rG = sum(self.r[..., c] * G[c] for c in range(3))
        out = [dh]
        for c in range(3):
            a_, b_ = (c + 1) % 3, (c + 2) % 3
            cor = self.fr[..., a_] * W[1 + b_] - self.fr[..., b_] * W[1 + a_]
            out.append(-self.g * (G[c] - self.r[..., c] * rG) - cor)
        return torch.stack(out)

    def dense_step(self, W: torch.Tensor, dt: float) -> torch.Tensor:
        W1 = W + dt * self.dense_rhs(W)
        W2 = 0.75 * W + 0.25 * (W1 + dt * self.dense_rhs(W1))
        return W / 3.0 + (2.0 / 3.0) * (W2 + dt * self.dense_rhs(W2))

    # ---- conversions / diagnostics --------------------------------------------
    def to_factored(self, W: torch.Tensor):
        """Factor a dense state (setup): the SVDs run on the host in fp64
        (LAPACK); rocSOLVER's device SVD left ~1e-9 relative errors in the
        initial factors, more than the whole factored run adds
        (profiles/r6_tt/README.md)."""
        def fac(U):
            f = LowRankField.from_dense(U.detach().to(device="cpu", dtype=torch.float64), min(self.eps, 1e-14),
                                        self.max_rank)
            return LowRankField(f.A.to(device=self.device, dtype=self.dtype),
                                f.B.to(device=self.device, dtype=self.dtype))
        return [[fac(W[q, p]) for p in range(6)] for q in range(4)]

    @staticmethod
    def to_dense(F) -> torch.Tensor:
        return torch.stack([torch.stack([f.dense() for f in Fq]) for Fq in F])

    def mass(self, W: torch.Tensor) -> float:
        return float((W[0] / self.invA).sum())

    def gaussian_hill(self, lon0: float = 0.3, lat0: float = 0.4, width: float = 0.25, amp: float = 10.0):
        """A resting layer with a Gaussian hill of height perturbation: the
        gravity waves it sheds cross every panel edge within a few hours."""
        c = self.grid.centers()
        p0 = np.array([math.cos(lat0) * math.cos(lon0), math.cos(lat0) * math.sin(lon0), math.sin(lat0)])
        d = np.arccos(np.clip(c @ p0, -1.0, 1.0))
        h = amp * np.exp(-(d / width) ** 2)
        W = np.zeros((4, 6, self.N, self.N))
        W[0] = h
        return torch.as_tensor(W, dtype=self.dtype, device=self.device)


def _cdiff(X: torch.Tensor, h: float) -> torch.Tensor:
    """Periodic central difference of a factor's rows, (X[i+1] - X[i-1]) / 2h."""
    return (torch.roll(X, -1, 0) - torch.roll(X, 1, 0)) * (0.5 / h)


class LowRankShallowWater:
    """Linearised rotating shallow water on a doubly periodic N x N square,
    carried entirely in factored form: the Cartesian 2-D SWEs the slides cite
    for the 124x TT speed-up (PDF s.3, LANL, Danis et al. 2024),
    the research target the reference's FV solver is the baseline for
    (PDF s.5, s.19).

        h_t = -H (u_x + v_y),   u_t = -g h_x + f v,   v_t = -g h_y - f u

    on a C-free collocated grid (rows y, columns x, spacing L / N), second-order
    central differences, SSP-RK3.  Every field is F = A B^T; x derivatives act
    on the column factor (A (D B)^T), y derivatives on the row factor
    ((D A) B^T), so the right-hand side of each field is a sum of two rank-r
    products and a stage is one concatenation of factors:

        L_h = [-H A_u, -H D A_v] [D B_u, B_v]^T
        L_u = [-g A_h,   f A_v ] [D B_h, B_v]^T
        L_v = [-g D A_h, -f A_u] [B_h,   B_u]^T

    followed by a recompression to ``eps`` (backend "torch": thin QRs + a k x k
    SVD; "hip": CholeskyQR3 of every factor on the gfx950 kernels, the three
    fields' cores in one host transfer, ``recompress_many``).  The scheme
    conserves the total of h exactly (periodic central differences) and the
    energy g h^2 / 2 + H (u^2 + v^2) / 2 up to the SSP-RK3 dissipation.
    ``dense_step`` is the N x N reference of the same discrete operator; the
    semi-discrete dispersion relation omega^2 = f^2 + g H (k_x'^2 + k_y'^2),
    k' = sin(k dx) / dx, is the analytic check (tests/test_tt_and_models.py)."""

    def __init__(self, N: int, L: float = 1.0, g: float = 1.0, H: float = 1.0, f: float = 0.0,
                 eps: float = 1e-12, max_rank: Optional[int] = None, dtype=torch.float64, device="cpu",
                 backend: str = "torch"):
        if backend not in ("torch", "hip"):
            raise ValueError(f"unknown backend {backend!r}")
        self.N, self.L, self.h = N, L, L / N
        self.g, self.H, self.f = g, H, f
        self.eps, self.max_rank, self.backend = eps, max_rank, backend
        self.dtype, self.device = dtype, torch.device(device)
        c = math.sqrt(g * H)
        self.dt_max = self.h / (c * math.sqrt(2.0) + abs(f) * self.h + 1e-300)
        self.stats = {"recompressions": 0, "max_k": 0}

    # ---- factored operator ----------------------------------------------------
    def rhs_factors(self, F):
        """Factors (A, B) of L_h, L_u, L_v (each two rank-r blocks)."""
        h_, u_, v_ = F
        H, g, f, dx = self.H, self.g, self.f, self.h
        Lh = (torch.cat([-H * u_.A, -H * _cdiff(v_.A, dx)], 1), torch.cat([_cdiff(u_.B, dx), v_.B], 1))
        Lu = (torch.cat([-g * h_.A, f * v_.A], 1), torch.cat([_cdiff(h_.B, dx), v_.B], 1))
        Lv = (torch.cat([-g * _cdiff(h_.A, dx), -f * u_.A], 1), torch.cat([h_.B, u_.B], 1))
        return [Lh, Lu, Lv]

    def _recompress(self, pairs) -> List[LowRankField]:
        self.stats["recompressions"] += 1
        self.stats["max_k"] = max(self.stats["max_k"], max(A.shape[1] for A, _ in pairs))
        if self.backend == "hip":
            return recompress_many([(A.contiguous(), B.contiguous()) for A, B in pairs], self.eps, self.max_rank,
                                   "hip")
        return [recompress(A, B, self.eps, self.max_rank) for A, B in pairs]

    def _combo(self, terms) -> List[LowRankField]:
        """sum_i a_i X_i (+ b L(Y)) per field, as one recompression of the
        concatenated factors.  terms: list of (coef, fields) or (coef, 'L', Lfactors)."""
        pairs = []
        for q in range(3):
            As, Bs = [], []
            for t in terms:
                if t[1] == "L":
                    As.append(t[0] * t[2][q][0])
                    Bs.append(t[2][q][1])
                else:
                    As.append(t[0] * t[1][q].A)
                    Bs.append(t[1][q].B)
            pairs.append((torch.cat(As, 1), torch.cat(Bs, 1)))
        return self._recompress(pairs)

    def step(self, F: Sequence[LowRankField], dt: float) -> List[LowRankField]:
        """One SSP-RK3 step of (h, u, v); three recompressions (one per stage)."""
        U1 = self._combo([(1.0, F), (dt, "L", self.rhs_factors(F))])
        U2 = self._combo([(0.75, F), (0.25, U1), (0.25 * dt, "L", self.rhs_factors(U1))])
        return self._combo([(1.0 / 3.0, F), (2.0 / 3.0, U2), (2.0 / 3.0 * dt, "L", self.rhs_factors(U2))])

    # ---- dense reference ---------------------------------------------------------
    def dense_rhs(self, W: torch.Tensor) -> torch.Tensor:
        """W [3, N, N] = (h, u, v), rows y, columns x."""
        h_, u_, v_ = W
        dx = self.h
        ddx = lambda X: (torch.roll(X, -1, 1) - torch.roll(X, 1, 1)) * (0.5 / dx)
        ddy = lambda X: (torch.roll(X, -1, 0) - torch.roll(X, 1, 0)) * (0.5 / dx)
        return torch.stack([-self.H * (ddx(u_) + ddy(v_)), -self.g * ddx(h_) + self.f * v_,
                            -self.g * ddy(h_) - self.f * u_])

    def dense_step(self, W: torch.Tensor, dt: float) -> torch.Tensor:
        W1 = W + dt * self.dense_rhs(W)
        W2 = 0.75 * W + 0.25 * (W1 + dt * self.dense_rhs(W1))
        return W / 3.0 + (2.0 / 3.0) * (W2 + dt * self.dense_rhs(W2))

    # ---- conversions / diagnostics ------------------------------------------------
    def to_factored(self, W: torch.Tensor) -> List[LowRankField]:
        return [LowRankField.from_dense(W[q].to(device=self.device, dtype=self.dtype), min(self.eps, 1e-14),
                                        self.max_rank) for q in range(3)]

    @staticmethod
    def to_dense(F: Sequence[LowRankField]) -> torch.Tensor:
        return torch.stack([f.dense() for f in F])

    def energy(self, W: torch.Tensor) -> float:
        h_, u_, v_ = W
        return float((0.5 * self.g * h_ * h_ + 0.5 * self.H * (u_ * u_ + v_ * v_)).sum() * self.h * self.h)

    def gravity_wave(self, kx: int, ky: int, amp: float = 0.1):
        """Initial state of one standing inertia-gravity mode (h = amp cos(kx x)
        cos(ky y), u = v = 0) and the semi-discrete frequency omega of the
        scheme's central differences: h(t) = h(0) (f^2 + g H k'^2 cos(omega t))
        / omega^2 for the rotating case."""
        N, L = self.N, self.L
        x = (torch.arange(N, dtype=torch.float64) + 0.5) * self.h
        ax, ay = 2 * math.pi * kx / L, 2 * math.pi * ky / L
        h0 = amp * torch.outer(torch.cos(ay * x), torch.cos(ax * x))
        W = torch.stack([h0, torch.zeros_like(h0), torch.zeros_like(h0)])
        kpx, kpy = math.sin(ax * self.h) / self.h, math.sin(ay * self.h) / self.h
        omega = math.sqrt(self.f ** 2 + self.g * self.H * (kpx ** 2 + kpy ** 2))
        return W.to(self.dtype), omega, (kpx, kpy)


def compress_cubed_sphere(field: np.ndarray, eps: float = 1e-6, qtt: bool = False) -> List[dict]:
    """Per-panel TT ranks, compression and error of a [6, N, N] field."""
    out = []
    for f in range(6):
        x = torch.as_tensor(field[f], dtype=torch.float64)
        t = qtt_reshape(x) if qtt else x
        cores = tt_svd(t, eps)
        rec = tt_full(cores)
        rec = qtt_unreshape(rec) if qtt else rec
        err = float(torch.linalg.norm(rec - x) / max(float(torch.linalg.norm(x)), 1e-300))
        out.append({"face": f, "ranks": tt_ranks(cores), "storage": tt_storage(cores),
                    "compression": x.numel() / tt_storage(cores), "rel_error": err})
    return out
