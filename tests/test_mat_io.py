"""`.mat` I/O: qmc_utils.load_data / load_mat / save_map against the
reference's shipped file (tests/golden/onebitdata1.mat, a byte copy of qmc/onebitdata1.mat) and
the fixture tools/make_golden.py wrote from it by the reference's own loader + the notebook's
permutes (tests/golden/mat_c1.npz; qmc/qmc_utils.py:12-20, qmc/qmc.ipynb:497-503)."""
import os

import numpy as np
import scipy.io as sio
import torch

from quantized_spectrum_cartography_amd import qmc_utils

MAT = os.path.join(os.path.dirname(__file__), "golden", "onebitdata1.mat")


def test_load_data_reference_layout():
    """permute=False is qmc_utils.load_data itself: MATLAB layout, float32."""
    S, C, T, S_true, C_true, T_true = qmc_utils.load_data(MAT)
    raw = sio.loadmat(MAT)
    for name, x in zip(("S", "C", "T", "S_true", "C_true", "T_true"),
                       (S, C, T, S_true, C_true, T_true)):
        assert x.dtype == torch.float32
        assert tuple(x.shape) == raw[name].shape
        assert np.array_equal(x.numpy(), raw[name].astype(np.float32))
    assert tuple(T.shape) == (51, 51, 64) and tuple(S_true.shape) == (51, 51, 2)
    assert tuple(C_true.shape) == (64, 2)


def test_load_data_permuted_matches_golden(golden):
    """permute=True reproduces mat_c1.npz (written from the reference's own load) bit-exactly."""
    g = golden("mat_c1")
    S, C, T, S_true, C_true, T_true = qmc_utils.load_data(MAT, permute=True)
    assert np.array_equal(S_true.numpy(), g["S_true"])
    assert np.array_equal(C_true.numpy(), g["C_true"])
    assert np.array_equal(T_true.numpy(), g["T_true"])
    assert np.array_equal(T.numpy().astype(np.int8), g["T"])
    assert tuple(S.shape) == (2, 51, 51) and tuple(C.shape) == (2, 64)
    assert not S.any() and not C.any()
    m = qmc_utils.load_mat(MAT)
    assert np.array_equal(m["Om"].numpy().astype(np.uint8), g["Om"])


def test_onebit_field_reproduces_shipped_T():
    """generate_test_data.m:63-66 applied to the file's T_true gives the file's T exactly."""
    raw = sio.loadmat(MAT, mat_dtype=True)
    assert np.array_equal(qmc_utils.onebit_field(raw["T_true"]), raw["T"])


def test_save_map_round_trip(tmp_path):
    """load_mat -> save_map -> load_mat is the identity on every variable, and the written file
    has generate_test_data.m's variable names, MATLAB classes and layout."""
    m = qmc_utils.load_mat(MAT)
    out = str(tmp_path / "roundtrip.mat")
    qmc_utils.save_map(out, m["T_true"], m["S_true"], m["C_true"], T=m["T"], Om=m["Om"])
    raw = sio.loadmat(out, mat_dtype=True)
    assert {"C", "T", "S", "C_true", "S_true", "Om", "T_true"} <= set(raw)
    assert raw["T"].shape == (51, 51, 64) and raw["S"].shape == (51, 51, 2)
    assert raw["C"].shape == (64, 2) and raw["Om"].dtype == bool
    m2 = qmc_utils.load_mat(out)
    for k in m:
        assert np.array_equal(m[k].numpy(), m2[k].numpy()), k
    # the permuted round trip reproduces the golden too
    S, C, T, S_true, C_true, T_true = qmc_utils.load_data(out, permute=True)
    ref = sio.loadmat(MAT)
    assert np.array_equal(T_true.permute(1, 2, 0).numpy(), ref["T_true"].astype(np.float32))


def test_save_map_defaults_threshold_and_mask(tmp_path):
    """Default T = the one-bit field, Om = round(f*I*J) sampled pixels (generate_test_data.m)."""
    g = torch.Generator().manual_seed(3)
    K, R, I, J = 16, 2, 9, 7
    S_true = torch.rand(R, I, J, generator=g) * 0.01
    C_true = torch.rand(R, K, generator=g)
    T_true = torch.einsum("rij,rk->kij", S_true, C_true)
    out = str(tmp_path / "gen.mat")
    qmc_utils.save_map(out, T_true, S_true, C_true, f=0.3, seed=1)
    m = qmc_utils.load_mat(out)
    assert int(m["Om"].sum()) == round(0.3 * I * J)
    expect = np.where(T_true.double().numpy() > qmc_utils.MEAN_SLF, 1.0, -1.0)
    assert np.array_equal(m["T"].double().numpy(), expect)
    prob = qmc_utils.onebit_problem_from_mat(out)
    assert prob["Y"].shape == (K, 1, I, J) and prob["Y"].dtype == torch.int64
    assert set(torch.unique(prob["Y"]).tolist()) <= {0, 1}
    assert torch.equal(prob["Wx"][3, 0].bool(), m["Om"])


def test_onebit_problem_from_shipped_mat(golden):
    """Config 1 one-bit variant from the file: the same Y, Wx, b the
    GPU fixture test builds from mat_c1.npz."""
    g = golden("mat_c1")
    prob = qmc_utils.onebit_problem_from_mat(MAT)
    Y = torch.from_numpy((g["T"].astype(np.int64) + 1) // 2).unsqueeze(1)
    assert torch.equal(prob["Y"], Y)
    assert torch.equal(prob["Wx"], torch.ones(64, 1, 51, 51))  # Om is all ones in the file
    assert prob["b"].tolist() == [0.0, np.float32(0.0045).item(), float(g["T_true"].max())]
    assert prob["R"] == 2
