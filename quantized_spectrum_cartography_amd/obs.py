"""Observation sets: the quantized, sparsely sampled map packed for the fused HIP passes.

The reference keeps the observation as a dense int64 tensor Y (K,1,I,J) plus a dense float
mask Wx (qmc/qmc.ipynb :493, :537) and evaluates every entry.  `Observations` folds the mask
into uint8 codes (0xFF = unobserved), then packs only the observed entries into the two
sliced formats of include/qsc.h (one per pass), with pixels re-ordered by observation count
so that the 64 lanes of every wavefront carry near-equal work.  Built once per solve.
"""
import os

import torch

from . import _lib
from ._model import _dev, _ws


def ctypes_copy(dst, src):
    """Field-by-field copy of a ctypes Structure."""
    for name, _ in src._fields_:
        setattr(dst, name, getattr(src, name))


def default_tile(P, R, K):
    """C-pass pixel tile (positions, a power of two in [256, 1024]; 128 at rank 16 when LDS
    requires it).

    The C-pass runs one 4-wave workgroup per (tile, 64-bin slice): aim for ~1024 workgroups
    (4 per CU) while keeping tiles large, since the per-bin lists of a tile are padded to their
    longest (bigger tiles -> relatively less padding) and the tile's S rows live in LDS.  At
    least 256 positions: the fused launch (one workgroup per tile) then runs two S-step slices
    per wave and its C-finish sums half as many tiles -- C2 (256^2 x 64) 131.4 k grad-steps/s
    at 256 against 129.8 k at 128 (profiles/r04/fin_small_wg/ab_c2*.log)."""
    if os.environ.get("QSC_CTILE"):  # tuning override (power of two, 64..4096)
        return int(os.environ["QSC_CTILE"])
    Pp = -(-P // 64) * 64
    nks = -(-K // 64)
    if R <= 8:
        # the tile-form C-pass and the fused launch run one workgroup per tile: ~256 tiles (one
        # round on the 256 CUs) whatever K is.  Sizing by tiles x k-slices (the per-slice C-pass
        # form's rule) gave the K-slab shares of C3 (K_loc = 32, 64) 256-position tiles and 4x
        # the slab rows to finish: c3k8 C-finish 6.87 us at 256 positions, 3.26 us at 1024, C-pass
        # 9.81 / 9.57 us (profiles/r06/kslab/c3k8_tiles.log)
        t = 256
        while t * 256 < Pp and t < 1024:
            t *= 2
        return t
    want = max(1, (Pp * nks) // 1024)
    t = 256
    while t * 2 <= want and t < 1024:
        t *= 2
    if R > 8:
        # rank 16: the fused S-step + C-pass launch holds C^T and the S tile at a 20-float
        # pitch in LDS (scfused_lds, qsc_pass.hip); halve the tile until both fit, with the
        # part-sum area of the largest part count it may use
        parts = 1 if nks >= 16 else 16 // nks
        part_sum = 16 * 64 * 4 * nks * parts if parts > 1 else 0
        while t > 128 and 32 + K * 80 + 2048 + t * 80 + part_sum + 64 > 160 * 1024:
            t //= 2
    return t


class Observations:
    """Packed observations of one K-slab.

    Args:
      Y: bin indices, (K,1,I,J) or (K,I,J) integer tensor (quantize output).
      Wx: sampling mask of the same shape (0/1 floats) or None (all observed).
      bin_boundaries, noise_std, offset, log_model: the probit model (see quantization_model*).
      perm: optional (Pp,) int32 pixel order shared across ranks (K-slab sharding).
      tile: optional C-pass tile size (positions, multiple of 64).
      loss: "probit" (the likelihood of qmc/qmc.ipynb) or "squared" (the Euclidean criterion
            ||Wx (T_hat - Obs)||^2 of qmc/qmc_dowjons.ipynb :142, Obs the bin midpoints).
      schedule: order every packed list for bank-conflict-free LDS gathers (qsc_obs_schedule;
            default on, QSC_SCHEDULE=0 turns it off).  Results change only by summation order.
    """

    def __init__(self, Y, Wx, bin_boundaries, noise_std, offset=0.0, log_model=False, perm=None,
                 tile=None, R_hint=8, count_hook=None, loss="probit", schedule=None):
        K = Y.shape[0]
        I, J = Y.shape[-2], Y.shape[-1]
        P = I * J
        if schedule is None:  # QSC_SCHEDULE=0: natural list order (A/B switch)
            schedule = os.environ.get("QSC_SCHEDULE", "1") != "0"
        self.schedule = bool(schedule)
        self.K, self.I, self.J, self.P = K, I, J, P
        PT = int(tile or default_tile(P, R_hint, K))
        if PT < 64 or PT % 64:
            raise ValueError("tile must be a positive multiple of 64")
        self.Pp = -(-P // PT) * PT  # whole tiles; padding positions carry no observations
        self.model = _lib.make_model(bin_boundaries, noise_std, offset if log_model else 0.0,
                                     log_model, loss=loss)
        self.loss = loss
        self.log_model = bool(log_model)
        self.noise_std = float(noise_std)
        self.offset = float(offset or 0.0)
        self.bin_boundaries = [float(x) for x in (bin_boundaries.tolist() if isinstance(
            bin_boundaries, torch.Tensor) else bin_boundaries)]
        nbins = len(self.bin_boundaries) - 1
        if nbins > 254:
            raise ValueError("at most 254 bins are supported (code 0xFF marks unobserved)")
        Yd = _dev(Y.reshape(K, P).to(torch.int64))
        dev = Yd.device
        self.device = dev
        Wd = _dev(Wx.reshape(K, P).to(torch.float32)) if Wx is not None else None
        codes = torch.empty((K, P), dtype=torch.uint8, device=dev)
        bad = torch.zeros(1, dtype=torch.int32, device=dev)
        _lib.call("qsc_pack_codes", _lib.ptr(Yd), _lib.ptr(Wd), K * P, nbins, _lib.ptr(codes),
                  _lib.ptr(bad), _lib.stream())
        nbad = int(bad.item())
        if nbad:
            raise ValueError("%d observed entries have a code outside [0, %d) or a sampling "
                             "weight other than 0/1" % (nbad, nbins))
        self.codes = codes
        s = _lib.stream()
        cnt = torch.empty(P, dtype=torch.int32, device=dev)
        _lib.call("qsc_obs_count", _lib.ptr(codes), K, P, _lib.ptr(cnt), s)
        self.counts = cnt
        if perm is None:
            # count_hook (e.g. an all-reduce over K-slab ranks) makes the pixel order a function
            # of the global counts, so every rank lays S out identically
            order_cnt = count_hook(cnt.clone()) if count_hook is not None else cnt
            perm = torch.empty(self.Pp, dtype=torch.int32, device=dev)
            ws = _ws(_lib.lib().qsc_obs_order_workspace_bytes(P), dev)
            _lib.call("qsc_obs_order", _lib.ptr(order_cnt), P, self.Pp, _lib.ptr(perm), _lib.ptr(ws),
                      ws.numel(), _lib.stream())
        else:
            perm = _dev(perm.to(torch.int32))
            if perm.numel() != self.Pp:
                raise ValueError("perm must have Pp = %d entries" % self.Pp)
        self.perm = perm
        ns, nt, nks = self.Pp // _lib.QSC_SLICE, self.Pp // PT, -(-K // 64)
        self.s_width = torch.empty(ns, dtype=torch.int32, device=dev)
        self.s_off = torch.empty(ns + 1, dtype=torch.int64, device=dev)
        self.c_width = torch.empty(nt * nks, dtype=torch.int32, device=dev)
        self.c_off = torch.empty(nt * nks + 1, dtype=torch.int64, device=dev)
        self.c_kmap = torch.empty(nt * nks * 64, dtype=torch.int32, device=dev)
        desc = _lib.QscObsDesc()
        ws = _ws(_lib.lib().qsc_obs_layout_workspace_bytes(K, P, PT), dev)
        _lib.call("qsc_obs_layout", _lib.ptr(codes), K, P, PT, nbins, _lib.ptr(perm), _lib.ptr(cnt),
                  _lib.ptr(self.s_width), _lib.ptr(self.s_off), _lib.ptr(self.c_width),
                  _lib.ptr(self.c_off), _lib.ptr(self.c_kmap), _lib.ptr(ws), ws.numel(), desc, s)
        self.desc = desc
        et = torch.int32 if desc.wide else torch.int16
        self.s_entries = torch.empty(desc.s_entries, dtype=et, device=dev)
        self.c_entries = torch.empty(desc.c_entries, dtype=et, device=dev)
        rowfmt = 1 if self.signed_rows_ok(R_hint) else 0
        desc.rowfmt = rowfmt
        # signed-row entries (include/qsc.h rowfmt 1: the one-bit kind reads each entry's code
        # through the gathered row) wherever the passes' doubled tables fit at this rank
        self._fill(rowfmt)

    def _fill(self, rowfmt, desc=None, s_entries=None, c_entries=None):
        """Pack the entries in format `rowfmt` into (desc, s_entries, c_entries) (default: this
        object's own arrays; only before any pass engine uses them, see layout())."""
        if desc is None:
            if getattr(self, "_engines", 0):
                raise RuntimeError("the packed entries are in use by a pass engine (and maybe a "
                                   "captured hipGraph): re-packing them in place is refused")
            desc, s_entries, c_entries = self.desc, self.s_entries, self.c_entries
        desc.rowfmt = int(rowfmt)
        _lib.call("qsc_obs_fill", _lib.ptr(self.codes), desc, _lib.ptr(self.perm),
                  _lib.ptr(self.s_width), _lib.ptr(self.s_off), _lib.ptr(self.c_width),
                  _lib.ptr(self.c_off), _lib.ptr(self.c_kmap), _lib.ptr(s_entries),
                  _lib.ptr(c_entries), _lib.stream())
        if self.schedule:
            # bank-conflict-free list order (include/qsc.h qsc_obs_schedule): the same order for
            # both entry formats (it depends only on the row residues), so their results agree
            ws = _ws(_lib.lib().qsc_obs_schedule_workspace_bytes(desc), self.device)
            _lib.call("qsc_obs_schedule", desc, _lib.ptr(self.s_width), _lib.ptr(self.s_off),
                      _lib.ptr(self.c_width), _lib.ptr(self.c_off), _lib.ptr(s_entries),
                      _lib.ptr(c_entries), _lib.ptr(ws), ws.numel(), _lib.stream())

    def signed_rows_ok(self, R):
        if os.environ.get("QSC_SIGNED_ROWS", "1") == "0":  # A/B switch (tuning runs)
            return False
        return bool(_lib.lib().qsc_obs_signed_rows_ok(self.desc, int(R), self.model))

    def layout(self, R):
        """(desc, s_entries, c_entries) the passes read at rank R.  The signed-row packing chosen
        for R_hint is used where it applies at R; otherwise a code-field copy is packed once and
        kept (same entry count, other values).  The shared packing is never re-packed in place,
        so hipGraphs captured by other solvers on this object stay valid (their kernels hold the
        descriptor and entry pointers by value)."""
        self._engines = getattr(self, "_engines", 0) + 1
        if self.desc.rowfmt != 1 or self.signed_rows_ok(R):
            return self.desc, self.s_entries, self.c_entries
        if getattr(self, "_code_field", None) is None:
            d = _lib.QscObsDesc()
            ctypes_copy(d, self.desc)
            s_e = torch.empty_like(self.s_entries)
            c_e = torch.empty_like(self.c_entries)
            self._fill(0, d, s_e, c_e)
            self._code_field = (d, s_e, c_e)
        return self._code_field

    # ---- info -----------------------------------------------------------------------
    @property
    def nnz(self):
        return int(self.desc.nnz)

    @property
    def entry_bytes(self):
        return 4 if self.desc.wide else 2

    def stats(self):
        d = self.desc
        return dict(K=d.K, P=d.P, Pp=d.Pp, tile=d.PT, ntiles=d.ntiles, nks=d.nks, wide=d.wide,
                    nbins=d.nbins, nnz=d.nnz, s_entries=d.s_entries, c_entries=d.c_entries,
                    rowfmt=d.rowfmt,
                    s_padding=d.s_entries / max(d.nnz, 1) - 1.0,
                    c_padding=d.c_entries / max(d.nnz, 1) - 1.0)

    # ---- order conversions -------------------------------------------------------------
    def rank_pad(self, R):
        """Row count RP of the position-order layout for rank R (4, 8 or 16)."""
        rp = int(_lib.lib().qsc_rank_pad(int(R)))
        if rp == 0:
            raise ValueError("rank R must be in [1, %d]" % _lib.QSC_MAX_R)
        return rp

    def iperm(self):
        """(P,) int32: the position of every pixel (inverse of perm; cached)."""
        ip = getattr(self, "_iperm", None)
        if ip is None:
            ip = torch.full((self.P,), -1, dtype=torch.int32, device=self.device)
            valid = self.perm >= 0
            ip[self.perm[valid].long()] = torch.arange(self.Pp, dtype=torch.int32,
                                                       device=self.device)[valid]
            self._iperm = ip
        return ip

    def to_positions(self, X, out=None):
        """(R, P) natural pixel order -> (Pp, RP) position order (pixel-major rows, zero padded);
        into `out` when given (a persistent buffer, e.g. inside a captured hipGraph)."""
        R = X.shape[0]
        Xd = _dev(X.detach().to(torch.float32)).reshape(R, self.P).contiguous()
        if out is None:
            out = torch.empty((self.Pp, self.rank_pad(R)), dtype=torch.float32, device=Xd.device)
        elif out.shape != (self.Pp, self.rank_pad(R)) or not out.is_contiguous():
            raise ValueError("out must be a contiguous (%d, %d) tensor" % (self.Pp, self.rank_pad(R)))
        _lib.call("qsc_perm_gather", _lib.ptr(Xd), _lib.ptr(self.perm), R, self.P, self.Pp,
                  _lib.ptr(out), _lib.stream())
        return out

    def to_pixels(self, Xp, R, out=None):
        """(Pp, RP) position order -> (R, P) natural pixel order."""
        if Xp.shape != (self.Pp, self.rank_pad(R)):
            raise ValueError("position-order tensor must be (%d, %d), got %s"
                             % (self.Pp, self.rank_pad(R), tuple(Xp.shape)))
        if out is None:
            out = torch.empty((R, self.P), dtype=torch.float32, device=Xp.device)
        _lib.call("qsc_perm_scatter", _lib.ptr(Xp.contiguous()), _lib.ptr(self.perm), R, self.P,
                  self.Pp, _lib.ptr(out), _lib.stream())
        return out
