"""Deep priors for the spatial loss fields S (torch modules; not part of the HIP hot path).

The reference's solver draws S from a generator network (qmc/qmc.ipynb :470-550):
  Generator256  deep_prior/networks/gan.py:83-126 — DCGAN-style z(256) -> 1x51x51 sigmoid
  DecoderDip    deep_prior/networks/dip.py:20-89 — Upsample+Conv+BN+SELU z(256) -> 1x51x51
The layer lists below keep the reference's module order so that state dicts saved by the
reference (key prefix `main.<index>`) load unchanged.  `SizedDecoderDip` generalises the DIP
decoder to other map sizes (e.g. 256x256 for config 5), which the reference cannot produce.
"""
import torch
import torch.nn as nn


class UnFlatten(nn.Module):
    def __init__(self, target_shape):
        super().__init__()
        self.target_shape = target_shape

    def forward(self, x):
        return torch.reshape(x, (x.size(0), *self.target_shape))


def _ct(cin, cout, k, s, p):
    return [nn.ConvTranspose2d(cin, cout, k, s, p), nn.BatchNorm2d(cout), nn.ReLU(True)]


class Generator256(nn.Module):
    """z (B,256) -> (B,1,51,51); sizes 1 -> 3 -> 6 -> 12 -> 26 -> 54 -> 51."""

    def __init__(self, ndf=16):
        super().__init__()
        layers = [UnFlatten((ndf * 16, 1, 1))]
        layers += _ct(ndf * 16, ndf * 8, 3, 1, 0)
        layers += _ct(ndf * 8, ndf * 4, 4, 2, 1)
        layers += _ct(ndf * 4, ndf * 2, 4, 2, 1)
        layers += _ct(ndf * 2, ndf, 4, 2, 0)
        layers += _ct(ndf, 2, 4, 2, 0)
        layers += [nn.Conv2d(2, 1, 4, 1, 0), nn.Sigmoid()]
        self.main = nn.Sequential(*layers)

    def forward(self, z):
        return self.main(z)


def _cbs(cin, cout, k, p):
    return [nn.Conv2d(cin, cout, k, 1, p), nn.BatchNorm2d(cout), nn.SELU()]


class DecoderDip(nn.Module):
    """z (B,256) -> (B,1,51,51); sizes 1 -> 2 -> 3 -> 6 -> 12 -> 26 -> 52 -> 51."""

    def __init__(self, ndf=16):
        super().__init__()
        up = lambda: nn.Upsample(scale_factor=2)  # noqa: E731
        L = [UnFlatten((ndf * 16, 1, 1)), up()]
        L += _cbs(ndf * 16, ndf * 8, 2, 1) + _cbs(ndf * 8, ndf * 8, 3, 1) + [up()]
        L += _cbs(ndf * 8, ndf * 4, 3, 1) + _cbs(ndf * 4, ndf * 4, 3, 1) + [up()]
        L += _cbs(ndf * 4, ndf * 2, 3, 1) + _cbs(ndf * 2, ndf * 2, 3, 1) + [up()]
        L += _cbs(ndf * 2, ndf, 3, 2) + _cbs(ndf, ndf, 3, 1) + [up()]
        L += _cbs(ndf, 2, 3, 1) + _cbs(2, 2, 3, 1)
        L += [nn.Conv2d(2, 1, 4, 1, 1), nn.Sigmoid()]
        self.main = nn.Sequential(*L)

    def forward(self, z):
        return self.main(z)


class SizedDecoderDip(nn.Module):
    """DecoderDip-style decoder for an arbitrary square map size.

    z (B, zdim) -> (B,1,size,size): 1x1 seed, then Upsample(x2) + two Conv3x3/BN/SELU blocks per
    octave until the map covers `size`, channels halving from 16*ndf down to 2, a 3x3 output conv
    with sigmoid, and a centre crop to `size`.
    """

    def __init__(self, size=256, zdim=256, ndf=16):
        super().__init__()
        self.size = size
        n_up = max(1, (size - 1).bit_length())
        ch = [max(2, (ndf * 16) >> i) for i in range(n_up + 1)]
        L = [UnFlatten((zdim, 1, 1))]
        cin = zdim
        for i in range(n_up):
            L += [nn.Upsample(scale_factor=2)]
            L += _cbs(cin, ch[i + 1], 3, 1) + _cbs(ch[i + 1], ch[i + 1], 3, 1)
            cin = ch[i + 1]
        L += [nn.Conv2d(cin, 1, 3, 1, 1), nn.Sigmoid()]
        self.main = nn.Sequential(*L)

    def forward(self, z):
        x = self.main(z)
        h = x.shape[-1]
        o = (h - self.size) // 2
        return x[..., o:o + self.size, o:o + self.size]
