"""CPU: the bank-conflict-free list order (csrc/qsc_sched.cuh) through its host form
qsc_sched_lists_host -- the same code the device pass qsc_obs_schedule runs per 16-lane group.

Checked: every lane keeps exactly its multiset of observed entries (the schedule only permutes
a list, so the passes sum the same terms), pads stay pads on the neutral rows, and in every slot
each row residue mod 16 (= LDS bank group of the gathered row) is read by at most
ceil(count / W) lanes -- once whenever the group has no more than W entries of that residue --
and pads take residues no entry of their slot reads.  Reference context: the C-step / S-step
gathers replace the dense get_tensor of qmc/qmc.ipynb :568-571, :626-629."""
import ctypes
from collections import Counter

import numpy as np
import pytest

from quantized_spectrum_cartography_amd import _lib


def _sched(lists, W, rowfmt, rows, wide=0):
    L = _lib.lib()
    a = np.ascontiguousarray(lists, dtype=np.uint32)
    out = np.zeros_like(a)
    rc = L.qsc_sched_lists_host(a.ctypes.data, out.ctypes.data, W, rowfmt, rows, wide)
    return rc, out


def _pad_base(rowfmt, rows, wide):
    if rowfmt:
        return 2 * ((rows + 15) // 16 * 16)
    return (255 << 24) if wide else (15 << 12)


def _is_pad(e, rowfmt, rows, wide):
    if rowfmt:
        return e >= _pad_base(rowfmt, rows, wide)
    return (e >> (24 if wide else 12)) == (255 if wide else 15)


def _random_lists(rng, W, rows, rowfmt, f, wide=0, skew=False):
    """16 lists in the natural packing: ascending row index, signed or code-field values, pads
    last (lengths drawn so the longest has W entries, as the width rounds up to it)."""
    so = (rows + 15) // 16 * 16
    out = np.zeros((16, W), np.uint32)
    lens = rng.binomial(W, f, 16).clip(0, W)
    lens[rng.integers(16)] = W
    for i in range(16):
        if skew:  # residues concentrated on a few values: forces 2-way splits
            pool = np.array([q for q in range(rows) if q % 16 in (0, 1, 5)])
        else:
            pool = np.arange(rows)
        n = min(lens[i], len(pool))
        idx = np.sort(rng.choice(pool, n, replace=False))
        code = rng.integers(0, 2, n)
        if rowfmt:
            vals = idx + code * so
        else:
            vals = idx | (code << (24 if wide else 12))
        out[i, :n] = vals
        out[i, n:] = _pad_base(rowfmt, rows, wide)
    return out


def _check(inp, out, W, rowfmt, rows, wide=0):
    real_in = [Counter(int(e) for e in inp[i] if not _is_pad(int(e), rowfmt, rows, wide)) for i in range(16)]
    real_out = [Counter(int(e) for e in out[i] if not _is_pad(int(e), rowfmt, rows, wide)) for i in range(16)]
    assert real_in == real_out, "a lane's entries changed"
    cnt = Counter(int(e) & 15 for i in range(16) for e in inp[i] if not _is_pad(int(e), rowfmt, rows, wide))
    bound = {r: max(1, -(-c // W)) for r, c in cnt.items()}
    worst = 1
    for c in range(W):
        col = [int(out[i, c]) for i in range(16)]
        reals = Counter(e & 15 for e in col if not _is_pad(e, rowfmt, rows, wide))
        pads = [e & 15 for e in col if _is_pad(e, rowfmt, rows, wide)]
        for r, m in reals.items():
            assert m <= bound[r], (c, r, m, bound[r])
            worst = max(worst, m)
        assert len(set(pads)) == len(pads), "pads of one slot share a residue"
        assert not set(pads) & set(reals), "a pad shares a residue with an entry of its slot"
        for e in col:
            if _is_pad(e, rowfmt, rows, wide):
                if rowfmt:
                    assert e - _pad_base(rowfmt, rows, wide) < 16  # one of the 16 pad rows
                else:
                    assert (e & ((1 << (24 if wide else 12)) - 1)) < rows
    return worst


@pytest.mark.parametrize("seed,W,rows,rowfmt,f", [
    (0, 104, 1024, 1, 0.93),   # C3 C-format block: ~100-entry lists over a 1024-position tile
    (1, 28, 256, 1, 0.9),      # C3 S-format slice group: ~26 entries over 256 bins
    (2, 32, 70, 1, 0.8),       # K not a multiple of 16 (negated half at round_up(K, 16))
    (3, 64, 512, 0, 0.7),      # code-field values
    (4, 8, 40, 1, 0.5),        # short lists
    (5, 256, 4096, 1, 0.95),   # the longest scheduled lists
    (6, 12, 13, 1, 0.9),       # fewer rows than residues
])
def test_schedule_is_a_conflict_free_permutation(seed, W, rows, rowfmt, f):
    rng = np.random.default_rng(seed)
    inp = _random_lists(rng, W, rows, rowfmt, f)
    rc, out = _sched(inp, W, rowfmt, rows)
    assert rc == 0
    _check(inp, out, W, rowfmt, rows)


def test_schedule_splits_overfull_residues_evenly():
    """A residue with more than W entries in the group is read at most ceil(count / W) times per
    slot (2-way at worst here), never more."""
    rng = np.random.default_rng(7)
    W, rows = 40, 512
    inp = _random_lists(rng, W, rows, 1, 0.95, skew=True)
    rc, out = _sched(inp, W, 1, rows)
    assert rc == 0
    worst = _check(inp, out, W, 1, rows)
    assert worst >= 2  # the skewed residues really exceed W ...


def test_schedule_wide_entries():
    rng = np.random.default_rng(8)
    W, rows = 48, 5000
    inp = _random_lists(rng, W, rows, 0, 0.8, wide=1)
    rc, out = _sched(inp, W, 0, rows, wide=1)
    assert rc == 0
    _check(inp, out, W, 0, rows, wide=1)


def test_long_lists_keep_natural_order():
    rng = np.random.default_rng(9)
    W, rows = 260, 4096
    inp = _random_lists(rng, W, rows, 1, 0.9)
    rc, out = _sched(inp, W, 1, rows)
    assert rc == 1 and np.array_equal(inp, out)


def test_all_pad_group():
    W, rows = 16, 256
    inp = np.full((16, W), _pad_base(1, rows, 0), np.uint32)
    rc, out = _sched(inp, W, 1, rows)
    assert rc == 0
    _check(inp, out, W, 1, rows)


def test_natural_order_has_conflicts_the_schedule_removes():
    """The natural ascending order of a C3-like block conflicts (several lanes per residue in a
    slot); the schedule brings every slot to one lane per residue."""
    rng = np.random.default_rng(10)
    W, rows = 104, 1024
    inp = _random_lists(rng, W, rows, 1, 0.93)

    def cycles(a):
        """mean LDS cycles of the slot's 16-lane ds_read_b128 group (max lanes per residue)"""
        return np.mean([max(Counter(int(e) & 15 for e in a[:, c]).values()) for c in range(W)])
    rc, out = _sched(inp, W, 1, rows)
    assert rc == 0 and _check(inp, out, W, 1, rows) <= 2
    assert cycles(inp) > 2.5 and cycles(out) < 1.35, (cycles(inp), cycles(out))
