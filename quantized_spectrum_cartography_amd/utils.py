"""Bin-boundary, noise and offset constants of the quantization models.

Values are the reference's data, re-stated so that existing callers find them under the same
names (qmc/utils.py:11-51).  The `*_ADJUSTED` edges and offsets are the output of the
Gauss-Newton offset fit of qmc/nlls.py, which this package reproduces in `nlls.fit_log_offset`
(checked against these constants in tests/test_oracle_golden.py).  The one-bit threshold
`MEAN_SLF` is deep_prior/slf_dataset.py:11 / qmc/generate_test_data.m:24.
"""
import torch

# equal-count bins of raw map values (qmc/utils.py:11-15)
QUANTIZATION_BOUNDARIES_8_BINS_SAMPLE = [0.0, 3.219041422308777e-10, 6.34243551758118e-05,
                                         0.0001823223865358159, 0.00036289551644586027,
                                         0.0006664704997092485, 0.0012639077613130212,
                                         0.00301913358271122, 0.3312782347202301]
SD_8_BINS_SAMPLE = 3.219041422308777e-10

QUANTIZATION_BOUNDARIES_16_BINS = [0.0, 8.944017748646615e-10, 2.3812383005861193e-05,
                                   6.808515900047496e-05, 0.00012131989933550358,
                                   0.00018234866729471833, 0.00025588355492800474,
                                   0.00034619917278178036, 0.0004588317824527621,
                                   0.0006049227667972445, 0.0007961964583955705,
                                   0.0010579598601907492, 0.001441714819520712,
                                   0.0020772861316800117, 0.003326504724100232,
                                   0.006930550094693899, 0.27432483434677124]
SD_16_BINS = 8.944017748646615e-10

# equally spaced bins over [0, 0.3312] (qmc/utils.py:18-25)
QUANTIZATION_BOUNDARIES_8_BINS_UNIFORM = torch.arange(9) * 0.3312 / 8
SD_8_BINS_UNIFORM = QUANTIZATION_BOUNDARIES_8_BINS_UNIFORM[1] - QUANTIZATION_BOUNDARIES_8_BINS_UNIFORM[0]
QUANTIZATION_BOUNDARIES_16_BINS_UNIFORM = torch.arange(17) * 0.3312 / 16
SD_16_BINS_UNIFORM = QUANTIZATION_BOUNDARIES_16_BINS_UNIFORM[1] - QUANTIZATION_BOUNDARIES_16_BINS_UNIFORM[0]
QUANTIZATION_BOUNDARIES_256_BINS_UNIFORM = torch.arange(257) * 0.3312 / 256
SD_256_BINS_UNIFORM = QUANTIZATION_BOUNDARIES_256_BINS_UNIFORM[1] - QUANTIZATION_BOUNDARIES_256_BINS_UNIFORM[0]

# equal-count bins of log map values (qmc/utils.py:29-35)
QUANTIZATION_BOUNDARIES_8_BINS_LOG = [-23.025850296020508, -23.000225067138672, -9.472214698791504,
                                      -8.490324974060059, -7.831082344055176, -7.240789890289307,
                                      -6.61128044128418, -5.762726783752441, -1.2379993200302124]
SD_8_BINS_LOG = 0.0256
QUANTIZATION_BOUNDARIES_7_BINS_LOG = [-23.025850296020508, -9.472214698791504, -8.490324974060059,
                                      -7.831082344055176, -7.240789890289307, -6.61128044128418,
                                      -5.762726783752441, -1.2379993200302124]
QUANTIZATION_BOUNDARIES_4_BINS_LOG = [-23.025850296020508, -10.002398490905762, -7.980128765106201,
                                      -6.692554473876953, -1.0331487655639648]
LOG_OFFSET_4 = 1e-10
SD_4_BINS_LOG = 1.287

# log(f + x) fitted edges and offsets (qmc/utils.py:43-51, produced by qmc/nlls.py)
QUANTIZATION_BOUNDARIES_7_ADJUSTED = [-10.69232977, -9.35950321, -8.49230102, -7.86067357,
                                      -7.27999497, -6.65573177, -5.7952887, -1.10472809]
QUANTIZATION_BOUNDARIES_16_ADJUSTED = [-15.25285591, -10.63537803, -9.59126825, -9.01512351,
                                       -8.60828803, -8.26986013, -7.96781035, -7.68630929,
                                       -7.41001714, -7.13536627, -6.85118837, -6.54175727,
                                       -6.17657863, -5.70576175, -4.97178181, -1.29344148]
LOG_OFFSET_7_ADJUSTED = 2.27e-05
LOG_OFFSET_16_ADJUSTED = 2.3755e-07

# one-bit threshold of the shipped fixture (qmc/generate_test_data.m:24, :65-66)
MEAN_SLF = 0.0045


def find_boundaries(samples, num_bins=4):
    """Equal-count bin edges of `samples` and the smallest bin width (qmc/utils.py:57-74).

    Walks the sorted values, closing a bin once it holds more than its share of points and the
    value strictly increased; the share is recomputed for the remaining bins after each edge.
    """
    data = torch.as_tensor(samples).reshape(-1).sort().values
    n = len(data)
    per_bin = int(n / num_bins)
    edges = [data[0].item()]
    count = 0
    for i in range(n):
        count += 1
        if count > per_bin and data[i] > edges[-1]:
            edges.append(data[i].item())
            per_bin = int((n - i) / (num_bins - len(edges) + 1))
            count = 0
    if not len(edges) > num_bins:
        edges.append(data[-1].item())
    sd = min(edges[i + 1] - edges[i] for i in range(len(edges) - 1))
    return edges, sd
