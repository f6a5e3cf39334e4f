"""ORACLE (test infrastructure only) — synthetic radio-map pieces in numpy fp64.

Restates qmc/generate_map.m:95-113 (path loss x log-normal shadowing, unit Frobenius norm,
optional dB) and qmc/Shadowing_data.m:1-25 (shadowing as the lower Cholesky factor of the full
exponential correlation matrix times i.i.d. N(0, var^2) draws) for small grids.  MATLAB is not
in this image, so there is no run of the reference to pin against: the compose step is
checked against this restatement on identical shadow inputs, and the shadowing generators
(this Cholesky form and the package's circulant embedding) against the analytic covariance
var^2 exp(-d / Xc) the reference's comment states (Shadowing_data.m:6-7).
"""
import numpy as np


def grid_distance(I, J, loc, res=1.0):
    """|Xgrid - location|, Xgrid = x + 1i*y with x along columns (meshgrid, generate_map.m:86-90)."""
    y, x = np.meshgrid(np.arange(I) * res, np.arange(J) * res, indexing="ij")
    return np.sqrt((x - loc[0]) ** 2 + (y - loc[1]) ** 2)


def compose(shadow, loc, alpha, res=1.0, d0=2.0, dB=False):
    shadow = np.asarray(shadow, np.float64)
    R, I, J = shadow.shape
    out = np.empty_like(shadow)
    for r in range(R):
        d = grid_distance(I, J, loc[r], res)
        with np.errstate(divide="ignore"):
            loss = np.minimum(1.0, (d / d0) ** (-float(alpha[r])))
        s = loss * 10.0 ** (shadow[r] / 10.0)
        s = s / np.linalg.norm(s)
        out[r] = np.real(10 * np.log10(s)) if dB else s
    return out


def shadowing_chol(I, J, var, Xc, rng, res=1.0):
    """Shadowing_data(Cloc, var, p = exp(-1/Xc)) for an I x J unit grid."""
    p = np.exp(-1.0 / Xc)
    y, x = np.meshgrid(np.arange(I) * res, np.arange(J) * res, indexing="ij")
    z = (x + 1j * y).reshape(-1, order="F")  # MATLAB column-major Cloc(:)
    D = np.abs(z[:, None] - z[None, :])
    Lc = np.linalg.cholesky(p ** D)
    iid = var * rng.standard_normal(I * J)
    return (Lc @ iid).reshape((I, J), order="F")


def exp_cov(d, var, Xc):
    return var ** 2 * np.exp(-np.asarray(d, np.float64) / Xc)
