"""bf16 MFMA GEMM (native/kernels/gemm.hip) — the Mars-style matmul map kernel.

:func:`matmul_tn` computes ``alpha · A · Btᵀ`` for bf16 ``A[M, K]`` and
``Bt[N, K]`` (K-contiguous operands) with fp32 accumulation on the CDNA4
matrix cores; any M and N (ragged edge tiles are zero-filled by the loads'
range check), K padded only to a multiple of 8.  On CPU it
falls back to a float32 torch matmul (CPU map slots).
"""
from __future__ import annotations

import torch

from . import _lib

TM, TN, TK = 256, 256, 64


def _pad(x: torch.Tensor, rows: int, cols: int) -> torch.Tensor:
    r, c = x.shape
    if r == rows and c == cols:
        return x.contiguous()
    out = torch.zeros(rows, cols, dtype=x.dtype, device=x.device)
    out[:r, :c] = x
    return out


def matmul_tn(a: torch.Tensor, bt: torch.Tensor, alpha: float = 1.0,
              out_dtype=torch.float32, stream=None, with_sum=False):
    """C = alpha · A · Btᵀ.  ``with_sum``: returns (C, fp64 sum of C's elements
    as stored), the sum taken in the GEMM epilogue (per-tile partials)."""
    if a.dim() != 2 or bt.dim() != 2 or a.shape[1] != bt.shape[1]:
        raise ValueError("A[M,K], Bt[N,K] required")
    M, K = a.shape
    N = bt.shape[0]
    if a.device.type != "cuda":
        c = ((a.float() @ bt.float().t()) * alpha).to(out_dtype)
        return (c, c.sum(dtype=torch.float64)) if with_sum else c
    if a.dtype != torch.bfloat16 or bt.dtype != torch.bfloat16:
        raise ValueError("bf16 operands required on the GPU")
    if out_dtype not in (torch.float32, torch.bfloat16):
        raise ValueError("C must be fp32 or bf16")
    # ragged M and N run natively (zero-filled edge tiles, masked stores); K
    # only needs whole 16-B pieces, so just a K % 8 tail is padded here
    Kp = -(-K // 8) * 8
    ap, bp = _pad(a, M, Kp), _pad(bt, N, Kp)
    if ap.data_ptr() % 16 or bp.data_ptr() % 16:
        ap, bp = ap.clone(), bp.clone()       # (views at odd offsets)
    c = torch.empty(M, N, dtype=out_dtype, device=a.device)
    part = torch.empty((-(-M // TM)) * (-(-N // TN)), dtype=torch.float64, device=a.device) \
        if with_sum else None
    rc = _lib.load().hbmr_gemm_bf16_tn_ex(ap.data_ptr(), bp.data_ptr(), c.data_ptr(), M, N, Kp,
                                           float(alpha), int(out_dtype == torch.bfloat16),
                                           part.data_ptr() if part is not None else None,
                                           _lib.stream_handle(stream))
    _lib.check(rc, "hbmr_gemm_bf16_tn_ex")
    return (c, part.sum()) if with_sum else c


def matmul(a: torch.Tensor, b: torch.Tensor, **kw) -> torch.Tensor:
    """A[M,K] · B[K,N] (transposes B once into the K-contiguous layout)."""
    return matmul_tn(a, b.t().contiguous(), **kw)
