"""Timing of the C4 (512 x 512 x 1024, R = 16) problem build steps in one process (diagnostic for
the multi-rank strong-scaling set-up)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from quantized_spectrum_cartography_amd import _model
    I, J, K, R = 512, 512, 1024, 16
    dev = "cuda"
    t = time.perf_counter()

    def lap(msg):
        nonlocal t
        torch.cuda.synchronize()
        now = time.perf_counter()
        print("%-28s %.2f s" % (msg, now - t), flush=True)
        t = now
    g = torch.Generator(device=dev).manual_seed(20263)
    S_true = torch.rand(R, 1, I, J, generator=g, device=dev)
    C_true = torch.rand(R, K, generator=g, device=dev)
    lap("rand S, C")
    T = _model.get_tensor(S_true, C_true)
    lap("get_tensor")
    thr2 = float(torch.sort(T.reshape(-1)).values[(T.numel() - 1) // 2])
    lap("median by sort")
    thr = float(T.median())
    lap("median")
    print("same value:", thr == thr2, flush=True)
    tmax, tmin = float(T.max()), float(T.min())
    lap("max/min")
    noise = torch.randn(T.shape, generator=g, device=dev)
    lap("randn")
    b = torch.tensor([0.0, thr, tmax])
    Y = _model.quantize(T, (tmax - tmin) / 4, b, noise=noise)
    lap("quantize")
    Wx = torch.bernoulli(torch.full((K, 1, I, J), 0.1, device=dev), generator=g)
    lap("bernoulli")
    del Y, Wx, noise, T


if __name__ == "__main__":
    main()
