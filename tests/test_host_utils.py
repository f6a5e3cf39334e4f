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
