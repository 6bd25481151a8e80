"""Plain-PyTorch reference implementations (no native code) of every operator.

They are the independent oracles of the numerics tests: fp32 for the image
operators (luminance, Roberts, KxK conv via ``torch.nn.functional.conv2d``),
fp64 for lab1/lab3/Jacobi. Summation order can differ from the native
kernels', so image results agree to +-1 gray level except where stated.
"""

from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from .filters import MODE_ABS1, MODE_MAG2, Filter


def luma(img: torch.Tensor) -> torch.Tensor:
    """fp32 luminance with the reference's evaluation order and no FMA."""
    f = img[..., :3].to(torch.float32)
    t0 = torch.tensor(0.299, dtype=torch.float32) * f[..., 0]
    t1 = torch.tensor(0.587, dtype=torch.float32) * f[..., 1]
    t2 = torch.tensor(0.114, dtype=torch.float32) * f[..., 2]
    return (t0 + t1) + t2


def _gray(g: torch.Tensor, alpha: torch.Tensor) -> torch.Tensor:
    v = torch.clamp(g, 0.0, 255.0).to(torch.uint8)  # truncating cast, like the reference
    return torch.stack([v, v, v, alpha], dim=-1)


def roberts(img: torch.Tensor) -> torch.Tensor:
    y = luma(img.cpu())
    yd = torch.cat([y[1:], y[-1:]], dim=0)  # clamp-to-edge neighbours
    yr = torch.cat([y[:, 1:], y[:, -1:]], dim=1)
    ydr = torch.cat([yd[:, 1:], yd[:, -1:]], dim=1)
    gx = ydr - y
    gy = yr - yd
    g = torch.sqrt(gx * gx + gy * gy)
    return _gray(g, img.cpu()[..., 3])


def roberts_rgb(img: torch.Tensor) -> torch.Tensor:
    """Per-channel Roberts cross, L1 magnitude, saturated; alpha kept."""
    x = img.cpu().to(torch.int32)
    xd = torch.cat([x[1:], x[-1:]], dim=0)
    xr = torch.cat([x[:, 1:], x[:, -1:]], dim=1)
    xdr = torch.cat([xd[:, 1:], xd[:, -1:]], dim=1)
    g = ((x - xdr).abs() + (xr - xd).abs()).clamp(max=255)
    g[..., 3] = x[..., 3]
    return g.to(torch.uint8)


def conv(img: torch.Tensor, filt: Filter) -> torch.Tensor:
    y = luma(img.cpu())
    up, down = filt.anchor, filt.k - 1 - filt.anchor
    yp = F.pad(y[None, None], (up, down, up, down), mode="replicate")
    dwx, dwy = filt.dense()  # separable filters: their K x K outer products, one direct sum
    wx = torch.tensor(dwx, dtype=torch.float32).reshape(1, 1, filt.k, filt.k)
    gx = F.conv2d(yp, wx)[0, 0]
    if filt.base_mode == MODE_MAG2:
        wy = torch.tensor(dwy, dtype=torch.float32).reshape(1, 1, filt.k, filt.k)
        gy = F.conv2d(yp, wy)[0, 0]
        g = torch.sqrt(gx * gx + gy * gy)
    elif filt.base_mode == MODE_ABS1:
        g = gx.abs()
    else:
        g = gx
    return _gray(g, img.cpu()[..., 3])


def vsub(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    return a.cpu() - b.cpu()


def classify_dist(img: torch.Tensor, mu: np.ndarray, inv: np.ndarray, device=None,
                  chunk: int = 1 << 21) -> torch.Tensor:
    """fp64 quadratic forms (p - mu_c)^T A_c (p - mu_c) of every pixel and class,
    (N, C), computed in pixel chunks (an 8192^2 image x 32 classes would need
    51 GB at once) on ``device`` (default: the CPU) with plain torch ops."""
    dev = torch.device(device) if device is not None else torch.device("cpu")
    p_all = img.reshape(-1, 4)[:, :3]
    m = torch.as_tensor(mu, dtype=torch.float64, device=dev)
    A = torch.as_tensor(inv, dtype=torch.float64, device=dev)
    out = torch.empty((p_all.shape[0], m.shape[0]), dtype=torch.float64)
    for s0 in range(0, p_all.shape[0], chunk):
        p = p_all[s0:s0 + chunk].to(dev).to(torch.float64)
        d = p[:, None, :] - m[None, :, :]  # (n, C, 3)
        t = torch.einsum("ncj,cji->nci", d, A)
        out[s0:s0 + chunk] = (t * d).sum(-1).cpu()
    return out


def classify(img: torch.Tensor, mu: np.ndarray, inv: np.ndarray, device=None) -> torch.Tensor:
    """fp64 direct quadratic forms, strict-< argmin (lowest class on ties), NaN -> 255."""
    dist = classify_dist(img, mu, inv, device)
    # a class is a candidate only if dist < DBL_MAX (NaN and +inf never win)
    cand = dist < torch.finfo(torch.float64).max
    d2 = torch.where(cand, dist, torch.full_like(dist, float("inf")))
    cls = torch.argmin(d2, dim=1)  # first minimum = lowest class index
    a = torch.where(cand.any(dim=1), cls, torch.full_like(cls, 255)).to(torch.uint8)
    out = img.cpu().clone().reshape(-1, 4)
    out[:, 3] = a
    return out.reshape(img.shape)


def jacobi(u: torch.Tensor, r0: int, r1: int) -> torch.Tensor:
    """One sweep over rows [r0, r1) (1-based, halo rows at 0 and rows+1)."""
    u = u.cpu().to(torch.float64)
    un = u.clone()
    c = u[r0:r1, 1:-1]
    s = ((u[r0 - 1:r1 - 1, 1:-1] + u[r0 + 1:r1 + 1, 1:-1]) + (u[r0:r1, :-2] + u[r0:r1, 2:])) * 0.25
    un[r0:r1, 1:-1] = s
    del c
    return un
