"""GPU: the device list schedule (qsc_obs_schedule, csrc/qsc_sched.cuh) on real packings.

Every list keeps its entries (a permutation per lane), the LDS gathers it induces are (near)
conflict-free in both formats, and the passes / solver give the oracle's results within the
north_star tolerance (1e-5) -- the schedule only changes summation order.  Reference: the
gathers stand in for the dense get_tensor of qmc/qmc.ipynb :568-571, :626-629."""
from collections import Counter

import numpy as np
import pytest
import torch

from conftest import rel_fro
from test_gpu_fused import _random_case

pytestmark = pytest.mark.gpu

GROUPS = [[0, 1, 2, 3, 12, 13, 14, 15] + list(range(20, 28)),
          list(range(4, 12)) + [16, 17, 18, 19, 28, 29, 30, 31]]
GROUPS += [[x + 32 for x in g] for g in GROUPS]


def _lists(obs, fmt):
    """{block: [per-lane entry lists]} read back from the device arrays (include/qsc.h)."""
    if fmt == "s":
        width, off, ent, lanes = obs.s_width, obs.s_off, obs.s_entries, 32
    else:
        width, off, ent, lanes = obs.c_width, obs.c_off, obs.c_entries, 64
    width = width.cpu().numpy()
    off = off.cpu().numpy()
    e = ent.cpu().numpy().astype(np.int64) & 0xFFFF
    out = []
    for b in range(len(width)):
        W = int(width[b])
        j = np.arange(W)
        rows = []
        for lane in range(lanes):
            idx = off[b] + (j // 4) * (lanes * 4) + lane * 4 + (j % 4)
            rows.append(e[idx])
        out.append(np.array(rows).reshape(lanes, W))
    return out


def _pad(obs, fmt, v):
    if obs.desc.rowfmt == 0:
        return (v >> 12) == 15
    rows = obs.K if fmt == "s" else obs.desc.PT
    so = (rows + 15) // 16 * 16
    return v >= 2 * so


def _cycles(obs, fmt, lists):
    """mean LDS cycles per 16-lane ds_read_b128 group and slot (max lanes sharing a residue)"""
    tot, n = 0, 0
    lanes = 32 if fmt == "s" else 64
    for L in lists:
        for g in GROUPS[: lanes // 16]:
            for c in range(L.shape[1]):
                tot += max(Counter(int(v) & 15 for v in L[g, c]).values())
                n += 1
    return tot / max(n, 1)


def test_schedule_permutes_lists_and_removes_conflicts():
    from quantized_spectrum_cartography_amd.obs import Observations
    d = _random_case(81, 8, 96, 80, 256)
    a = Observations(d["Y"], d["Wx"], d["b"], d["sigma"], R_hint=8, schedule=False)
    b = Observations(d["Y"], d["Wx"], d["b"], d["sigma"], R_hint=8, schedule=True)
    assert a.desc.rowfmt == b.desc.rowfmt == 1
    for fmt in ("s", "c"):
        la, lb = _lists(a, fmt), _lists(b, fmt)
        for A, B in zip(la, lb):
            for lane in range(A.shape[0]):
                ra = Counter(int(v) for v in A[lane] if not _pad(a, fmt, v))
                rb = Counter(int(v) for v in B[lane] if not _pad(b, fmt, v))
                assert ra == rb
        ca, cb = _cycles(a, fmt, la), _cycles(b, fmt, lb)
        # S-format groups hold whole pixel lists (~26 entries over 16 residues in W ~ 28
        # slots), so more residues exceed W than in the C-format's ~100-entry bin lists
        assert ca > 2.0 and cb < (1.75 if fmt == "s" else 1.5), (fmt, ca, cb)


@pytest.mark.parametrize("R,I,J,K,tile", [(8, 96, 80, 256, None), (4, 64, 64, 64, 512),
                                          (3, 50, 70, 130, 256), (16, 64, 64, 128, 512)])
def test_scheduled_solver_matches_natural_order(R, I, J, K, tile):
    """Solver S, C after 9 iterations with and without the schedule: equal to fp32 summation
    order (1e-5 relative Frobenius, the north_star tolerance), fused launch in both."""
    from quantized_spectrum_cartography_amd import qmc
    from quantized_spectrum_cartography_amd.obs import Observations
    d = _random_case(82 + R, R, I, J, K)
    res = []
    for sch in (False, True):
        o = Observations(d["Y"], d["Wx"], d["b"], d["sigma"], R_hint=R, tile=tile, schedule=sch)
        r = qmc.solve(d["Y"], d["Wx"], d["b"], d["sigma"], S_init=d["S0"], C_init=d["C0"],
                      max_iter=9, obs=o)
        res.append(r)
    assert rel_fro(res[1].S.cpu().numpy(), res[0].S.cpu().numpy()) < 1e-5
    assert rel_fro(res[1].C.cpu().numpy(), res[0].C.cpu().numpy()) < 1e-5
    assert np.allclose(res[1].costs_s, res[0].costs_s, rtol=1e-5)
