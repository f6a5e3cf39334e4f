"""Scalable synthetic radio maps: qmc/generate_map.m + qmc/Shadowing_data.m on the GPU.

Reference (MATLAB, text only):
  generate_map.m:11-77   emitter power spectra: Gaussian (or squared-sinc) PSD bumps, the first
                         at bin 5 + (r-1) (separable) or 5 + r, two more at random bins of
                         10:2:K-2, plus (separable) one at bin 20; columns normalised
  generate_map.m:79-113  spatial loss fields: min(1, (d/d0)^-alpha) path loss (d0 = 2,
                         alpha ~ U[2, 2.5]) times log-normal shadowing 10^(shadow/10) with
                         E[z(x) z(x')] = sigma^2 exp(-|x - x'| / Xc); each field unit-norm
  generate_map.m:114-131 optional dB fields; X = sum_r Sc_r (x) c_r
  Shadowing_data.m:1-25  shadowing by a Cholesky factor of the full (IJ x IJ) correlation
                         matrix: O((IJ)^3), unusable beyond ~64 x 64 pixels.
MI355X design: the shadowing field is drawn by circulant embedding -- the exponential
covariance on a torus of at least twice the grid, eigenvalues by one FFT, fields by one more
(rocFFT through torch.fft), two independent fields per complex FFT -- O(IJ log IJ); path loss x
shadowing, the per-field norms and the normalisation run in one HIP kernel pair
(libqsc_hip.so: qsc_map_compose); the map is qsc_reconstruct (get_tensor).  Random draws use
numpy / torch generators seeded by the caller (MATLAB's mt19937ar streams are not reproduced).
"""
import math

import numpy as np
import torch

from . import _lib
from ._model import _dev, _ws, get_tensor


def psd_basis(K, R, rng, basis="g", separable=True):
    """Emitter spectra C_true (K, R), unit-norm columns (generate_map.m:11-77)."""
    if K < 14:
        raise ValueError("generate_map needs K >= 14 (PSD peaks at 10:2:K-2)")
    k = np.arange(1, K + 1, dtype=np.float64)
    if basis == "g":
        def Sx(f0, s):
            return np.exp(-(k - f0) ** 2 / (2 * s ** 2))
    else:
        def Sx(f0, a):
            x = (k - f0) / a
            return np.sinc(x) ** 2 * (np.abs(x) <= 1)
    ind_psd = np.arange(10, K - 1, 2)
    npk = 3
    cols = []
    shared = None if separable else rng.choice(ind_psd, npk - 1, replace=False)
    for rr in range(1, R + 1):
        peaks = rng.choice(ind_psd, npk - 1, replace=False) if separable else shared
        am = 0.5 + 1.5 * rng.random(npk)
        if separable:
            c = am[0] * Sx(5 + (rr - 1), 2 + 3 * rng.random())
        else:
            c = am[0] * Sx(5 + rr, 2 + 2 * rng.random())
        for q in range(1, npk):  # MATLAB am(q), q = 1..npk-1 (am(1) is reused)
            c = c + am[q - 1] * Sx(peaks[q - 1], 2 + 2 * rng.random())
        if separable:  # "for experiment": one more bump at bin 20 with the last am(q)
            c = c + am[npk - 2] * Sx(20, 2 + 2 * rng.random())
        cols.append(c)
    C = np.stack(cols, axis=1)
    n = np.linalg.norm(C, axis=0)
    return C / np.where(n == 0, 1.0, n)


def _embedding(I, J, Xc, res, device):
    """Eigenvalues of the exponential covariance exp(-d / Xc) on the smallest power-of-two
    torus of at least twice the grid (clipped at 0), and the clipped fraction."""
    M = 1 << max(1, (2 * I - 1).bit_length())
    N = 1 << max(1, (2 * J - 1).bit_length())
    m = torch.arange(M, device=device, dtype=torch.float64)
    n = torch.arange(N, device=device, dtype=torch.float64)
    dm = torch.minimum(m, M - m)[:, None] * res
    dn = torch.minimum(n, N - n)[None, :] * res
    c = torch.exp(-torch.sqrt(dm ** 2 + dn ** 2) / Xc)
    lam = torch.fft.fft2(c).real
    neg = float(lam.clamp(max=0).abs().sum() / lam.abs().sum())
    return lam.clamp(min=0), M, N, neg


def shadowing(I, J, sigma, Xc, n, generator=None, res=1.0, device="cuda"):
    """n independent shadowing fields (n, I, J) in dB with E[z(x) z(x')] = sigma^2
    exp(-|x - x'| / Xc) (Shadowing_data.m with p = exp(-1/Xc), generate_map.m:101)."""
    dev = torch.device(device)
    if sigma == 0:
        return torch.zeros((n, I, J), device=dev)
    lam, M, N, _ = _embedding(I, J, float(Xc), float(res), dev)
    amp = torch.sqrt(lam / (M * N)).to(torch.float32)
    out = []
    for _ in range((n + 1) // 2):
        xi = torch.randn((2, M, N), generator=generator).to(dev)
        Z = torch.fft.fft2(torch.complex(xi[0], xi[1]) * amp)
        out += [Z.real[:I, :J], Z.imag[:I, :J]]
    return (float(sigma) * torch.stack(out[:n])).contiguous()


def compose(shadow, loc, alpha, res=1.0, d0=2.0, dB=False, return_norms=False):
    """Unit-norm spatial loss fields (R, I, J) from shadowing fields (R, I, J) [dB], emitter
    locations loc (R, 2) = (x, y) and path-loss exponents alpha (R,) (generate_map.m:95-113)."""
    sd = _dev(shadow.detach().to(torch.float32))
    R, I, J = sd.shape
    ld = _dev(torch.as_tensor(loc, dtype=torch.float32).reshape(R, 2))
    ad = _dev(torch.as_tensor(alpha, dtype=torch.float32).reshape(R))
    S = torch.empty_like(sd)
    norms = torch.empty(R, dtype=torch.float32, device=sd.device)
    ws = _ws(_lib.lib().qsc_map_compose_workspace_bytes(R, I, J), sd.device)
    _lib.call("qsc_map_compose", _lib.ptr(sd), _lib.ptr(ld), _lib.ptr(ad), R, I, J, float(res),
              float(d0), 1 if dB else 0, _lib.ptr(S), _lib.ptr(norms), _lib.ptr(ws), ws.numel(),
              _lib.stream())
    return (S, norms) if return_norms else S


def generate_map(K, R, shadow_sigma=5.0, Xc=50.0, basis="g", separable=True, I=51, J=51,
                 dB=False, seed=None, res=1.0, device="cuda"):
    """generate_map(dB, K, R, shadow_sigma, Xc, structured_c, basis, separable) on an I x J
    grid (the reference's is 51 x 51, gridLen 50).  Returns dict(T (K, I, J) map, S (R, I, J)
    loss fields, C (R, K) spectra, peaks (R, 2) emitter pixel coordinates, locations, alpha)."""
    rng = np.random.default_rng(seed)
    gen = torch.Generator().manual_seed(int(rng.integers(1 << 62)))
    C = psd_basis(K, R, rng, basis, separable)  # (K, R)
    ext_x, ext_y = (J - 1) * res, (I - 1) * res
    loc = np.stack([ext_x * rng.random(R), ext_y * rng.random(R)], axis=1)  # 50*rand(s)
    alpha = 2 + 0.5 * rng.random(R)
    shadow = shadowing(I, J, shadow_sigma, Xc, R, gen, res, device)
    S = compose(shadow, loc, alpha, res, 2.0, dB)
    Ct = torch.from_numpy(C.T.astype(np.float32)).to(S.device).contiguous()
    T = get_tensor(S.reshape(R, 1, I, J), Ct)
    peaks = np.stack([np.clip(np.rint(loc[:, 0]), 0, 255), np.clip(np.rint(loc[:, 1]), 0, 255)],
                     axis=1).astype(np.uint8)  # uint8(real/imag(location))
    return {"T": T, "S": S, "C": Ct, "peaks": peaks, "locations": loc, "alpha": alpha}
