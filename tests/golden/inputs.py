"""Seeded synthetic inputs shared by the fixture generator and the GPU tests."""
import torch


def fp8_inputs(rows, cols, dtype, seed):
    """Log-normal row magnitudes + edge rows: zero row (clamp floor), subnormal-range row,
    exact fp8 grid values, outliers, a negative zero."""
    g = torch.Generator().manual_seed(seed)
    w = torch.randn(rows, cols, generator=g) * torch.exp(torch.randn(rows, 1, generator=g))
    w = w * 0.05
    if rows >= 6:
        w[0] = 0.0
        w[1] = torch.randn(cols, generator=g) * 1e-6
        w[2, :16] = torch.tensor([0.5, 0.625, 1.0, 448.0, -448.0, 0.001953125, 3.0, -2.5,
                                  1.125, 1.0625, 240.0, 224.0, 232.0, 0.0, -0.0, 17.0])
        w[3, 5] = 30.0
        w[4, 1] = -0.0
    return w.to(dtype)
