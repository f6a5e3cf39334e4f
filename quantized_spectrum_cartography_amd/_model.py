"""GPU implementations of the reference's quantization-model functions.

Shared by quantization_model.py (linear model, qmc/quantization_model.py) and
quantization_model_log.py (log-domain model, qmc/quantization_model_log.py).  Every function
takes and returns torch tensors; tensors on the CPU are moved to the current GPU for the HIP
kernel and the result is returned on the caller's device, so notebook-style code runs
unchanged.  Autograd is supported through explicit HIP backward kernels.
"""
import math

import torch

from . import _lib

_F32 = torch.float32


def _dev(t):
    """Move t to the current GPU (the kernels never run on the CPU)."""
    if not torch.cuda.is_available():
        raise _lib.QscError("no GPU visible: quantized_spectrum_cartography_amd runs its "
                            "hot path only as HIP kernels on MI355X (gfx950)")
    t = t if t.is_cuda else t.cuda()
    _lib.require_device(t)
    return t.contiguous()


def _ws(nbytes, device):
    return torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=device)


# ---------------------------------------------------------------------------------------
# quantize
# ---------------------------------------------------------------------------------------
def quantize(X, noise_std, bin_boundaries, offset=None, log_model=False, noise=None):
    """Bin index of X + N(0, std^2) (linear) or log(X + offset) + N(0, std^2) (log model).

    Reference: qmc/quantization_model.py:8-20, qmc/quantization_model_log.py:9-21.  The noise is
    drawn exactly as the reference draws it, `torch.randn(X.shape)` from torch's global CPU
    generator, so the same seed gives byte-identical Y; pass `noise` to supply it explicitly.
    Linear model: x = X + noise*std and the binning on the GPU (qsc_quantize).  Log model: x is
    formed on the host with torch's log, binned on the GPU (qsc_bin_codes), see there.
    """
    out_dev = X.device
    if log_model:
        # the reference log model's default offset (qmc/quantization_model_log.py:7, :9)
        from .utils import LOG_OFFSET_7_ADJUSTED
        offset = LOG_OFFSET_7_ADJUSTED if offset is None else float(offset)
        if not offset > 0.0:
            raise ValueError("the log model needs offset > 0 (log(X + offset) at X = 0)")
    if noise is None:
        noise = torch.randn(X.shape)
    if log_model:
        # x = log(X + offset) + randn*std formed with torch's CPU log, the reference's own op
        # (qmc/quantization_model_log.py:14): ocml's logf differs from ATen's vectorised log by
        # an ulp on some inputs, which would flip bin indices at edges.  Binning on the GPU.
        x = torch.log(X.detach().cpu().to(_F32) + offset) + noise.cpu().to(_F32) * noise_std
        xd = _dev(x)
        m = _lib.make_model(bin_boundaries, noise_std, offset, log_model)
        Y = torch.empty(xd.shape, dtype=torch.int64, device=xd.device)
        _lib.call("qsc_bin_codes", _lib.ptr(xd), xd.numel(), m, _lib.ptr(Y), _lib.stream())
        return Y.to(out_dev)
    Xd = _dev(X.to(_F32))
    nd = _dev(noise.to(_F32))
    m = _lib.make_model(bin_boundaries, noise_std, offset if log_model else 0.0, log_model)
    Y = torch.empty(Xd.shape, dtype=torch.int64, device=Xd.device)
    _lib.call("qsc_quantize", _lib.ptr(Xd), _lib.ptr(nd), Xd.numel(), m, _lib.ptr(Y), _lib.stream())
    return Y.to(out_dev)


# ---------------------------------------------------------------------------------------
# prob_probit (autograd w.r.t. X_hat)
# ---------------------------------------------------------------------------------------
class _ProbProbit(torch.autograd.Function):
    @staticmethod
    def forward(ctx, Y, X_hat, model):
        Yd, Xd = _dev(Y.to(torch.int64)), _dev(X_hat.to(_F32))
        Yd, Xd = torch.broadcast_tensors(Yd, Xd)
        Yd, Xd = Yd.contiguous(), Xd.contiguous()
        P = torch.empty(Xd.shape, dtype=_F32, device=Xd.device)
        _lib.call("qsc_prob_probit", _lib.ptr(Yd), _lib.ptr(Xd), Xd.numel(), model, _lib.ptr(P),
                  _lib.stream())
        ctx.model = model
        ctx.save_for_backward(Yd, Xd)
        ctx.x_shape = X_hat.shape
        return P

    @staticmethod
    def backward(ctx, gP):
        Yd, Xd = ctx.saved_tensors
        gP = gP.to(_F32).contiguous()
        gX = torch.empty_like(Xd)
        _lib.call("qsc_prob_probit_bwd", _lib.ptr(Yd), _lib.ptr(Xd), _lib.ptr(gP), Xd.numel(),
                  ctx.model, _lib.ptr(gX), _lib.stream())
        if gX.shape != ctx.x_shape:
            gX = gX.sum_to_size(ctx.x_shape)
        return None, gX, None


def prob_probit(Y, X_hat, bin_boundaries, noise_std, log_model=False):
    """P(Y | X_hat) = F(b[Y+1] - X_hat) - F(b[Y] - X_hat) under the probit model.

    Reference: qmc/quantization_model.py:22-39 (linear: b[0], b[-1] clamped to -/+1e5) and
    qmc/quantization_model_log.py:23-41 (log model: edges unclamped).
    """
    model = _lib.make_model(bin_boundaries, noise_std, 0.0, log_model)
    out_dev = X_hat.device
    P = _ProbProbit.apply(Y, X_hat, model)
    return P if out_dev.type == "cuda" else P.to(out_dev)


def F_probit(y, std):
    """0.5*(1 + erf(y/(std*1.414213))) (qmc/quantization_model.py:57-61, constant kept verbatim)."""
    yd = _dev(y.to(_F32))
    out = torch.empty_like(yd)
    _lib.call("qsc_f_probit", _lib.ptr(yd), yd.numel(), float(std), _lib.ptr(out), _lib.stream())
    return out.to(y.device)


def F_sigmoid(y):
    """1/(1+exp(-y)) (qmc/quantization_model.py:41-45)."""
    return torch.sigmoid(y)


def dither_probit(y, std):
    """Bernoulli sample with success probability F_probit(y, std) (qmc/quantization_model.py:63-68)."""
    return torch.bernoulli(F_probit(y, std))


def dither_sigmoid(y):
    """Bernoulli sample with success probability sigmoid(y) (qmc/quantization_model.py:47-53)."""
    return torch.bernoulli(F_sigmoid(y))


def get_quantized_obs_from_ordinal(Y, bin_boundaries, noise_std=None):
    """Mid-bin value (b[Y] + b[Y+1]) / 2 (qmc/quantization_model_log.py:43-51)."""
    Yd = _dev(Y.to(torch.int64))
    m = _lib.make_model(bin_boundaries, 1.0 if noise_std is None else noise_std)
    out = torch.empty(Yd.shape, dtype=_F32, device=Yd.device)
    _lib.call("qsc_obs_from_ordinal", _lib.ptr(Yd), Yd.numel(), m, _lib.ptr(out), _lib.stream())
    return out.to(Y.device)


# ---------------------------------------------------------------------------------------
# reconstruction T = sum_r S_r (x) c_r  (autograd through both factors)
# ---------------------------------------------------------------------------------------
class _GetTensor(torch.autograd.Function):
    @staticmethod
    def forward(ctx, S, C):
        R = S.shape[0]
        I, J = S.shape[-2], S.shape[-1]
        K = C.shape[1]
        Sd = _dev(S.to(_F32)).reshape(R, I * J)
        Cd = _dev(C.to(_F32)).reshape(R, K)
        T = torch.empty((K, I, J), dtype=_F32, device=Sd.device)
        _lib.call("qsc_reconstruct", _lib.ptr(Sd), _lib.ptr(Cd), R, I * J, K, _lib.ptr(T),
                  _lib.stream())
        ctx.save_for_backward(Sd, Cd)
        ctx.s_shape = S.shape
        return T

    @staticmethod
    def backward(ctx, gT):
        Sd, Cd = ctx.saved_tensors
        R, P = Sd.shape
        K = Cd.shape[1]
        gT = gT.to(_F32).contiguous()
        need_s, need_c = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        dS = torch.empty_like(Sd) if need_s else None
        dC = torch.empty_like(Cd) if need_c else None
        nb = _lib.lib().qsc_reconstruct_bwd_workspace_bytes(R, P, K)
        ws = _ws(nb, Sd.device)
        _lib.call("qsc_reconstruct_bwd", _lib.ptr(gT), _lib.ptr(Sd), _lib.ptr(Cd), R, P, K,
                  _lib.ptr(dS), _lib.ptr(dC), _lib.ptr(ws), ws.numel(), _lib.stream())
        return (dS.reshape(ctx.s_shape) if dS is not None else None), dC


def get_tensor(S, C):
    """sum_r S[r] (x) C[r] -> (K, I, J) (qmc/quantization_model.py:79-86).

    The r-sum runs in the reference's order with separately rounded products and sums, so the
    output is bit-identical to the reference's slice-by-slice accumulation.
    """
    if S.dim() == 3:
        S = S.unsqueeze(1)
    if S.shape[0] > _lib.QSC_MAX_R:
        raise ValueError("rank R=%d exceeds the supported maximum %d" % (S.shape[0], _lib.QSC_MAX_R))
    out_dev = S.device
    T = _GetTensor.apply(S, C)
    return T if out_dev.type == "cuda" else T.to(out_dev)


def outer(mat, vec):
    """vec (x) mat -> (len(vec), *mat.shape) (qmc/quantization_model.py:70-77)."""
    return get_tensor(mat.reshape(1, 1, *mat.shape[-2:]), vec.reshape(1, -1))


# ---------------------------------------------------------------------------------------
# NMSE / NMSE_LOG
# ---------------------------------------------------------------------------------------
def _diff_sumsq(T, T_target, use_log, offset):
    a = _dev(T.detach().to(_F32)).reshape(-1)
    b = _dev(T_target.detach().to(_F32)).reshape(-1)
    if a.numel() != b.numel():
        a, b = torch.broadcast_tensors(a.reshape(T.shape), b.reshape(T_target.shape))
        a, b = a.contiguous().reshape(-1), b.contiguous().reshape(-1)
    out = torch.empty(2, dtype=torch.float64, device=a.device)
    ws = _ws(_lib.lib().qsc_reduce_workspace_bytes(a.numel()), a.device)
    _lib.call("qsc_diff_sumsq", _lib.ptr(a), _lib.ptr(b), a.numel(), int(use_log), float(offset),
              _lib.ptr(out), _lib.ptr(ws), ws.numel(), _lib.stream())
    return out


def NMSE(T, T_target):
    """||T - T_target||_F / ||T_target||_F  (qmc/quantization_model.py:88-92; not squared)."""
    s = _diff_sumsq(T, T_target, False, 0.0)
    return (s[0].sqrt() / s[1].sqrt()).to(_F32).to(T.device)


def NMSE_LOG(T, T_target, offset):
    """NMSE of log(T + offset) vs log(T_target + offset) (qmc/quantization_model_log.py:104-111)."""
    s = _diff_sumsq(T, T_target, True, offset)
    return (s[0].sqrt() / s[1].sqrt()).to(_F32).to(T.device)


def map_nmse(S, C, T_true, log_offset=None):
    """NMSE(get_tensor(S, C), T_true) without materialising the reconstructed map."""
    R = S.shape[0]
    P = S.shape[-1] * S.shape[-2] if S.dim() >= 3 else S.shape[-1]
    K = C.shape[1]
    Sd = _dev(S.detach().to(_F32)).reshape(R, P)
    Cd = _dev(C.detach().to(_F32))
    Td = _dev(T_true.detach().to(_F32)).reshape(K, P)
    out = torch.empty(2, dtype=torch.float64, device=Sd.device)
    ws = _ws(_lib.lib().qsc_reduce_workspace_bytes(0), Sd.device)
    _lib.call("qsc_map_diff_sumsq", _lib.ptr(Sd), _lib.ptr(Cd), _lib.ptr(Td), R, P, K,
              int(log_offset is not None), float(log_offset or 0.0), _lib.ptr(out), _lib.ptr(ws),
              ws.numel(), _lib.stream())
    return math.sqrt(out[0].item()) / math.sqrt(out[1].item())


# ---------------------------------------------------------------------------------------
# BCE-probit likelihood and the deterministic cost
# ---------------------------------------------------------------------------------------
class NegLikelihood(torch.nn.Module):
    """BCE(mean) of F_probit(T - mean, std) (or sigmoid) against a {0,1} target.

    Reference: qmc/quantization_model.py:97-113 (the free-S solver's criterion,
    backup/notebooks/onebit_lowrank.ipynb:1238).
    """

    def __init__(self, mean, std=None, probit=True):
        super().__init__()
        self.mean = mean
        if probit:
            assert std is not None
        self.std = std
        self.probit = probit
        self.criterion = torch.nn.BCELoss()

    def forward(self, T_sample, T_target):
        if self.probit:
            z = T_sample - self.mean
            p = _FProbitAG.apply(z, self.std)
        else:
            p = F_sigmoid(T_sample - self.mean)
        return self.criterion(p, T_target.to(p.device))


class _FProbitAG(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, std):
        yd = _dev(y.to(_F32))
        out = torch.empty_like(yd)
        _lib.call("qsc_f_probit", _lib.ptr(yd), yd.numel(), float(std), _lib.ptr(out), _lib.stream())
        ctx.save_for_backward(yd)
        ctx.std = std
        return out

    @staticmethod
    def backward(ctx, g):
        (yd,) = ctx.saved_tensors
        a = float(torch.tensor(ctx.std * 1.414213, dtype=_F32))
        z = yd / a
        return g * torch.exp(-z * z) * (1.0 / (a * math.sqrt(math.pi))), None


class DeterministicCost(torch.nn.Module):
    """-lambda * <T_hat - mean, T_target> + ||T_hat - mean||_F (qmc/quantization_model.py:115-129)."""

    def __init__(self, mean=0):
        super().__init__()
        self.lambda_reg = 0.001
        self.mean = mean

    def forward(self, S, C, T_target):
        T_hat = get_tensor(S, C) - self.mean
        return -self.lambda_reg * (T_hat * T_target.to(T_hat.device)).sum() + torch.norm(T_hat, "fro")
