"""CPU: host-side bin-edge design (quantized_spectrum_cartography_amd.nlls / utils) against the
reference's own outputs (tests/golden/nlls.npz from running qmc/nlls.py; the qmc/utils.py:43-51
constants) and the oracle restatement."""
import numpy as np
import pytest
import torch

from oracle import nlls as onlls
from quantized_spectrum_cartography_amd import nlls, utils


def test_fit_log_offset_matches_reference_outputs(golden):
    g = golden("nlls")
    f, c, edges = nlls.fit_log_offset(g["raw"])
    assert np.allclose([f, c], g["theta"], rtol=1e-12, atol=0)
    assert np.allclose(edges, g["util_edges16"], rtol=0, atol=5e-8)
    th, e = onlls.gauss_newton(g["raw"])
    assert np.array_equal(edges, e) and (f, c) == tuple(th)


def test_adjusted_constants_reproduced():
    raw7 = [0.0, 6.34243551758118e-05, 0.0001823223865358159, 0.00036289551644586027,
            0.0006664704997092485, 0.0012639077613130212, 0.00301913358271122, 0.3312782347202301]
    f, _, e = nlls.fit_log_offset(raw7)
    assert abs(f - utils.LOG_OFFSET_7_ADJUSTED) / utils.LOG_OFFSET_7_ADJUSTED < 1e-3
    assert np.allclose(e, utils.QUANTIZATION_BOUNDARIES_7_ADJUSTED, atol=5e-8)


def test_design_log_bins_equal_count():
    g = torch.Generator().manual_seed(0)
    x = torch.rand(20000, generator=g) ** 4 * 0.3
    edges, f, raw, sd = nlls.design_log_bins(x, num_bins=8)
    assert len(raw) == 9 and len(edges) == 9 and f > 0
    counts = np.histogram(x.numpy(), bins=raw)[0]
    assert counts.min() > 0.8 * len(x) / 8
    # the fitted log edges are close to equally spaced (the purpose of the fit)
    d = np.diff(edges[1:-1])
    assert np.all(d > 0)


def test_log_quantize_rejects_nonpositive_offset():
    """quantize(log_model=True) validates the offset before any device work."""
    import torch
    from quantized_spectrum_cartography_amd._model import quantize
    X = torch.rand(2, 3, 3)
    b = torch.tensor([-30.0, -2.0, 0.0, 2.0])
    for off in (0.0, -1e-3):
        with pytest.raises(ValueError):
            quantize(X, 1.0, b, offset=off, log_model=True, noise=torch.zeros(X.shape))


def test_every_package_module_imports():
    """Import-level check of every module of the package (no GPU needed to import)."""
    import importlib
    import pkgutil
    import quantized_spectrum_cartography_amd as pkg
    for m in pkgutil.iter_modules(pkg.__path__):
        if m.name.startswith("libqsc"):  # (the HIP libraries, loaded through ctypes)
            continue
        importlib.import_module("%s.%s" % (pkg.__name__, m.name))


def _fin_arrive(ctr, t, nt, nvb, G_max=8):
    """The fused-finish arrival protocol of fin_arrive (csrc/qsc_pass.hip), restated: tile t
    counts on its group's counter (group g = t mod G, G = min(8, nt), n_g tiles); the group's
    last arrival counts the group complete; the last q_g arrivals of group g run C-finish items
    g, g + G, ... once the completed-group count reaches (launch + 1) G.  Counters are 64-bit and
    count for the life of the workspace.  Returns (item or -1, wait target or None)."""
    G = min(G_max, nt)
    g = t % G
    ng = (nt - g + G - 1) // G
    qg = (nvb - g + G - 1) // G if g < nvb else 0
    tk = ctr[g]
    ctr[g] += 1
    a, launch = tk % ng, tk // ng
    if a == ng - 1:
        ctr["groups"] += 1
    if a + qg < ng:
        return -1, None
    return g + G * (a + qg - ng), (launch + 1) * G


def test_fused_finish_ticket_protocol():
    """Every launch's C-finish items are each taken exactly once, by workgroups that wait for the
    same completed-group count, which is reached exactly when the launch's last tile arrives;
    any arrival order, any tile count >= R*nks + 2, consecutive launches (counters count up for
    the life of the workspace, from any start)."""
    import random
    rng = random.Random(5)
    for nt, nvb in ((256, 34), (64, 6), (34, 34), (36, 34), (1000, 130), (5, 3), (512, 6)):
        G = min(8, nt)
        for start_launch in (0, 7, 10 ** 12):
            ctr = {g: start_launch * ((nt - g + G - 1) // G) for g in range(G)}
            ctr["groups"] = start_launch * G
            for launch in range(3):
                order = list(range(nt))
                rng.shuffle(order)
                roles, done_at = [], None
                for i, t in enumerate(order):
                    roles.append(_fin_arrive(ctr, t, nt, nvb))
                    if done_at is None and ctr["groups"] >= (start_launch + launch + 1) * G:
                        done_at = i
                assert sorted(vb for vb, _ in roles if vb >= 0) == list(range(nvb))
                assert {w for vb, w in roles if vb >= 0} == {(start_launch + launch + 1) * G}
                # the waiters' count is reached exactly at the launch's last arrival
                assert done_at == nt - 1
                assert ctr["groups"] == (start_launch + launch + 1) * G


def test_split_holdout_partitions_the_observed_entries():
    """qmc.split_holdout: the fit and held-out masks partition the observed entries, the
    held-out share is about `frac`, and the split is a function of the seed."""
    import torch
    from quantized_spectrum_cartography_amd.qmc import split_holdout
    g = torch.Generator().manual_seed(3)
    Y = torch.zeros(16, 1, 20, 20, dtype=torch.int64)
    Wx = torch.bernoulli(torch.full((16, 1, 20, 20), 0.3), generator=g)
    a, b = split_holdout(Y, Wx, 0.1, seed=7)
    assert torch.equal(a + b, Wx) and torch.all(a * b == 0)
    frac = float(b.sum() / Wx.sum())
    assert 0.07 < frac < 0.13
    a2, b2 = split_holdout(Y, Wx, 0.1, seed=7)
    assert torch.equal(b, b2)
    _, b3 = split_holdout(Y, None, 0.1, seed=7)
    assert float(b3.mean()) > 0.07
