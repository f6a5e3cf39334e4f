"""GPU: the K-slab S-update kernels (reduce-scatter of dS -> Adam on the owned
1/N of S -> all-gather) against the whole-S update they replace.

qsc_supdate_slices applied shard by shard, with each shard's gradient handed over as its own
buffer (what the reduce-scatter delivers), must equal qsc_supdate on the whole S bit for bit --
S, Adam moments and the per-slice ||S_new||^2 partials -- and qsc_slice_nsq must rebuild those
partials from the gathered S exactly, so every rank settles the same regulariser norm.
Reference step: the S-step Adam of qmc/qmc.ipynb :622-634."""
import numpy as np
import pytest
import torch

from test_gpu_fused import _random_case

pytestmark = pytest.mark.gpu


def _setup(R=8, seed=91):
    from quantized_spectrum_cartography_amd import _lib
    from quantized_spectrum_cartography_amd.fused import PassEngine
    from quantized_spectrum_cartography_amd.obs import Observations
    d = _random_case(seed, R, 64, 80, 96)
    obs = Observations(d["Y"], d["Wx"], d["b"], d["sigma"], R_hint=R, tile=512)
    S = obs.to_positions(d["S0"].reshape(R, -1))
    g = torch.Generator(device="cpu").manual_seed(seed)
    dS = (torch.randn(S.shape, generator=g) * 0.1).cuda()
    dS[:, R:] = 0.0
    mS = (torch.randn(S.shape, generator=g) * 0.01).cuda()
    vS = (torch.rand(S.shape, generator=g) * 1e-4).cuda()
    mS[:, R:] = 0.0
    vS[:, R:] = 0.0
    adam = _lib.make_adam(1e-2, (0.9, 0.999), 1e-8, project_nonneg=False)
    return obs, S, dS, mS, vS, adam, R, PassEngine


@pytest.mark.parametrize("nshards", [1, 2, 3, 8])
def test_shard_updates_equal_whole_update(nshards):
    obs, S, dS, mS, vS, adam, R, PassEngine = _setup()
    a = PassEngine(obs, R)
    b = PassEngine(obs, R)
    a.init_state(S)
    b.init_state(S)
    Sa, ma, va = S.clone(), mS.clone(), vS.clone()
    Sb, mb, vb = S.clone(), mS.clone(), vS.clone()
    a.supdate(Sa, ma, va, dS, adam, 100.0)
    a.flush()
    Pp, u = obs.Pp, 32
    ns = Pp // u
    cs = -(-ns // nshards)
    for g in range(nshards):
        s0, s1 = min(g * cs, ns), min((g + 1) * cs, ns)
        g_own = dS[s0 * u:s1 * u].clone()  # the shard's reduce-scattered gradient, own buffer
        b.supdate_rows(Sb, mb, vb, g_own, adam, 100.0, s0 * u, s1 * u)
    b.slice_nsq(Sb)
    b.flush()
    torch.cuda.synchronize()
    for x, y in ((Sa, Sb), (ma, mb), (va, vb)):
        assert torch.equal(x, y)
    sa, sb = a.read_state(), b.read_state()
    assert sa["normsq_s"] == sb["normsq_s"] and sa["step_s"] == sb["step_s"] == 1


def test_slice_nsq_rebuilds_the_update_partials():
    obs, S, dS, mS, vS, adam, R, PassEngine = _setup(R=5, seed=92)
    a = PassEngine(obs, R)
    a.init_state(S)
    a.supdate(S, mS, vS, dS, adam, 100.0)
    torch.cuda.synchronize()
    n0 = a.ws.clone()  # the partials live in the pass workspace
    a.slice_nsq(S)
    torch.cuda.synchronize()
    assert torch.equal(n0, a.ws)


def test_adam_moments_flush_denormals_documented_deviation():
    """The pass library runs with f32 denormals flushed (the one-bit tail saturation relies on
    it), and its fused Adam epilogues share the setting: moments in the denormal
    range (|m| < 2^-126) are read and written as 0, where torch.optim.Adam on the CPU would keep
    them.  This pins the deviation; it cannot move S: an update of such a moment is
    below 1e-30 * lr, far under one ulp of any S value the solver carries."""
    obs, S, dS, mS, vS, adam, R, PassEngine = _setup(R=4, seed=93)
    e = PassEngine(obs, R)
    e.init_state(S)
    mS[:, :R] = 1e-39          # denormal
    vS[:, :R] = 1e-39
    dS.zero_()
    S0 = S.clone()
    e.supdate(S, mS, vS, dS, adam, 0.0)
    torch.cuda.synchronize()
    assert torch.count_nonzero(mS).item() == 0 and torch.count_nonzero(vS).item() == 0
    assert torch.equal(S, S0)


@pytest.mark.parametrize("R,tile", [(8, 512), (5, 512), (3, 256), (16, 512)])
def test_cpass_nsq_writes_the_slice_partials(R, tile):
    """qsc_cpass_nsq (the K-slab C-pass) leaves the workspace exactly as qsc_cpass followed by
    qsc_slice_nsq does -- dC slab, NLL partials, ||C||^2 slot and every slice's ||S||^2
    partial -- and the ||C||^2 slot (qsc_pass_cnsq_offset) holds qsc_sumsq_small's value."""
    from quantized_spectrum_cartography_amd.fused import PassEngine
    from quantized_spectrum_cartography_amd.obs import Observations
    d = _random_case(94 + R, R, 64, 80, 96)
    obs = Observations(d["Y"], d["Wx"], d["b"], d["sigma"], R_hint=R, tile=tile)
    S = obs.to_positions(d["S0"].reshape(R, -1))
    C = d["C0"].reshape(R, -1).cuda().contiguous()
    a, b = PassEngine(obs, R), PassEngine(obs, R)
    a.cpass(S, C)
    a.slice_nsq(S)
    b.cpass_nsq(S, C)
    torch.cuda.synchronize()
    assert torch.equal(a.ws, b.ws)
    ref = torch.zeros(1, device="cuda")
    a.sumsq(C, ref)
    torch.cuda.synchronize()
    assert torch.equal(b.cnsq(), ref)
