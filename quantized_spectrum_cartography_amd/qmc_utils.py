"""`.mat` I/O of the solver's data (qmc/qmc_utils.py, qmc/generate_test_data.m).

Reference behaviour restated here (text of the reference, not its code):
  qmc/qmc_utils.py:12-20     load_data(): scipy.io.loadmat of '../backup/data/onebitdata1', then
                             S, T, C, S_true, C_true, T_true as float32 torch tensors in MATLAB's
                             own layout: T, T_true (I, J, K); S, S_true (I, J, R); C, C_true (K, R)
  qmc/qmc.ipynb:497-503      the notebook permutes them for the solver: T(K, I, J), S(R, I, J),
                             C(R, K) ("compatibility with matlab generated arrays")
  qmc/generate_test_data.m:63-80
                             the writer: T = T_true with T(T<0) = 0, then T(T > mean_slf) = 1 and
                             T(T < mean_slf) = -1 (mean_slf = 0.0045; an entry exactly at
                             mean_slf keeps its value), the pixel mask Om (I, J) logical with
                             round(f*I*J) pixels drawn by randperm, zero S (I, J, R) and
                             C (K, R), saved as 'C', 'T', 'S', 'C_true', 'S_true', 'Om', 'T_true'.

This is host I/O only: the arrays go to the device with the solver (qmc.solve); nothing on the
hot path runs here.  MATLAB's randperm stream is not reproduced (numpy's generator draws Om).
"""
import numpy as np
import torch

MEAN_SLF = 0.0045  # qmc/generate_test_data.m:24 (the one-bit threshold), deep_prior mean_slf

_VARS = ("S", "C", "T", "S_true", "C_true", "T_true")


def _f32(a):
    return torch.from_numpy(np.ascontiguousarray(a)).type(torch.float32)


def _path(path):
    return str(path)


def load_data(path="../backup/data/onebitdata1", permute=False):
    """qmc/qmc_utils.py:12-20: (S, C, T, S_true, C_true, T_true), float32 tensors.

    permute=False returns the reference's own MATLAB layout (T (I, J, K), S (I, J, R),
    C (K, R)); permute=True applies the notebook's permutes (qmc/qmc.ipynb:497-503) and returns
    T (K, I, J), S (R, I, J), C (R, K) -- the solver's layout.  `path` is passed to
    scipy.io.loadmat as the reference does (the '.mat' suffix is optional)."""
    import scipy.io as sio
    data = sio.loadmat(_path(path))
    S, T, C = _f32(data["S"]), _f32(data["T"]), _f32(data["C"])
    S_true, C_true, T_true = _f32(data["S_true"]), _f32(data["C_true"]), _f32(data["T_true"])
    if permute:
        T, T_true = T.permute(2, 0, 1), T_true.permute(2, 0, 1)
        S, S_true = S.permute(2, 0, 1), S_true.permute(2, 0, 1)
        C, C_true = C.permute(1, 0), C_true.permute(1, 0)
    return S, C, T, S_true, C_true, T_true


def load_mat(path):
    """Every variable of a generate_test_data.m file in the solver's layout, plus the pixel mask
    (which load_data leaves out): dict(S (R, I, J), C (R, K), T (K, I, J), S_true, C_true,
    T_true, Om (I, J) bool), float32 tensors (Om a bool tensor)."""
    import scipy.io as sio
    data = sio.loadmat(_path(path))
    S, C, T, S_true, C_true, T_true = load_data(path, permute=True)
    out = dict(S=S, C=C, T=T, S_true=S_true, C_true=C_true, T_true=T_true)
    if "Om" in data:
        out["Om"] = torch.from_numpy(np.ascontiguousarray(data["Om"]).astype(bool))
    return out


def onebit_field(T_true, mean_slf=MEAN_SLF):
    """generate_test_data.m:63-66 on a (..) array: negatives to 0, then +1 above mean_slf and -1
    below it; an entry exactly equal to mean_slf is left as it is (MATLAB's two strict masks)."""
    T = np.array(T_true, dtype=np.float64, copy=True)
    T[T < 0] = 0
    T[T > mean_slf] = 1
    T[T < mean_slf] = -1
    return T


def sample_mask(I, J, f, rng):
    """generate_test_data.m:69-76: Om (I, J) logical with round(f*I*J) pixels, drawn without
    replacement (MATLAB linear indices are column-major, so the mask is filled in that order)."""
    IJ = I * J
    n = int(np.floor(f * IJ + 0.5))  # MATLAB round() rounds halves away from zero
    Ov = np.zeros(IJ, dtype=bool)
    Ov[rng.permutation(IJ)[:n]] = True
    return Ov.reshape((I, J), order="F")


def _np64(x):
    if isinstance(x, torch.Tensor):
        x = x.detach().cpu().numpy()
    return np.asarray(x, dtype=np.float64)


def save_map(path, T_true, S_true, C_true, f=1.0, mean_slf=MEAN_SLF, T=None, Om=None, seed=None):
    """Write a map in generate_test_data.m's variables and layout (qmc/generate_test_data.m:80).

    Inputs are in the solver's layout: T_true (K, I, J), S_true (R, I, J) or (R, 1, I, J),
    C_true (R, K) -- torch tensors or arrays (e.g. maps.generate_map's T, S, C).  T defaults to
    the one-bit field of T_true (onebit_field), Om to a sampled mask of round(f*I*J) pixels.
    Everything is stored as MATLAB doubles (Om as logical), transposed to T (I, J, K),
    S (I, J, R), C (K, R), with the zero initialisations S, C the script writes."""
    import scipy.io as sio
    Tt = _np64(T_true)
    K, I, J = Tt.shape
    St = _np64(S_true).reshape(-1, I, J)
    R = St.shape[0]
    Ct = _np64(C_true).reshape(R, K)
    Tq = onebit_field(Tt, mean_slf) if T is None else _np64(T).reshape(K, I, J)
    if Om is None:
        Om = sample_mask(I, J, f, np.random.default_rng(seed))
    Om = np.asarray(Om.cpu() if isinstance(Om, torch.Tensor) else Om).astype(bool).reshape(I, J)
    mdict = {
        "C": np.zeros((K, R)),
        "T": np.ascontiguousarray(Tq.transpose(1, 2, 0)),
        "S": np.zeros((I, J, R)),
        "C_true": np.ascontiguousarray(Ct.T),
        "S_true": np.ascontiguousarray(St.transpose(1, 2, 0)),
        "Om": Om,
        "T_true": np.ascontiguousarray(Tt.transpose(1, 2, 0)),
    }
    sio.savemat(_path(path), mdict, do_compression=True)
    return path


def onebit_problem_from_mat(path, sigma=0.02, mean_slf=MEAN_SLF):
    """Config 1's one-bit variant from a generate_test_data.m file:
    Y = (T + 1) / 2 in {0, 1} (K, 1, I, J) int64, the file's mask Om broadcast over K as Wx,
    the linear model's edges b = [0, mean_slf, max T_true] and the given sigma."""
    m = load_mat(path)
    K, I, J = m["T"].shape
    Y = ((m["T"].to(torch.int64) + 1) // 2).unsqueeze(1)
    Om = m.get("Om")
    Wx = (torch.ones(K, 1, I, J) if Om is None
          else Om.to(torch.float32).reshape(1, 1, I, J).expand(K, 1, I, J).contiguous())
    b = torch.tensor([0.0, float(mean_slf), float(m["T_true"].max())])
    R = m["S_true"].shape[0]
    return dict(Y=Y, Wx=Wx, b=b, sigma=float(sigma), R=R, S_true=m["S_true"].unsqueeze(1),
                C_true=m["C_true"], T_true=m["T_true"], log_model=False, offset=0.0)
