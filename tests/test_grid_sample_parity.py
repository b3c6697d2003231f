"""grid_sample / affine_grid against the reference's numpy oracles
(python/paddle/fluid/tests/unittests/test_grid_sampler_op.py GridSampler / AffineGrid, re-stated)."""
import numpy as np
import pytest

import paddle_hackathon_amd as paddle

R = np.random.RandomState(3)


def affine_grid_np(theta, n, h, w):
    h_idx = np.repeat(np.linspace(-1, 1, h)[None, :], w, axis=0).T[:, :, None]
    w_idx = np.repeat(np.linspace(-1, 1, w)[None, :], h, axis=0)[:, :, None]
    grid = np.concatenate([w_idx, h_idx, np.ones([h, w, 1])], axis=2)
    return np.stack([grid.reshape(h * w, 3) @ theta[i].T for i in range(n)]).reshape(n, h, w, 2)


def _unnorm(g, mx, align, pad):
    g = 0.5 * ((g + 1.0) * mx) if align else 0.5 * ((g + 1.0) * (mx + 1)) - 0.5
    if pad == "border":
        g = np.clip(g, 0, mx)
    elif pad == "reflection":
        dr = 2 * mx if align else (mx + 1) * 2
        ga = np.abs(g) if align else np.abs(g + 0.5)
        extra = ga - np.floor(ga / dr) * dr
        g = np.minimum(extra, dr - extra)
        g = g if align else np.clip(g - 0.5, 0, mx)
    return g


def _pt(data, x, y):
    N, C, H, W = data.shape
    out = np.zeros((N, C) + x.shape[1:])
    for i in range(N):
        ok = (x[i] >= 0) & (x[i] <= W - 1) & (y[i] >= 0) & (y[i] <= H - 1)
        xi, yi = np.clip(x[i], 0, W - 1), np.clip(y[i], 0, H - 1)
        out[i] = data[i][:, yi, xi] * ok
    return out


def grid_sample_np(data, grid, align, mode, pad):
    N, C, H, W = data.shape
    x = _unnorm(grid[..., 0], W - 1, align, pad)
    y = _unnorm(grid[..., 1], H - 1, align, pad)
    if mode == "nearest":
        return _pt(data, np.round(x).astype(int), np.round(y).astype(int))
    x0, y0 = np.floor(x).astype(int), np.floor(y).astype(int)
    x1, y1 = x0 + 1, y0 + 1
    w = lambda a: a[:, None]  # noqa: E731
    return (w((x1 - x) * (y1 - y)) * _pt(data, x0, y0) + w((x1 - x) * (y - y0)) * _pt(data, x0, y1) +
            w((x - x0) * (y1 - y)) * _pt(data, x1, y0) + w((x - x0) * (y - y0)) * _pt(data, x1, y1))


def test_affine_grid():
    theta = R.uniform(-1, 1, (2, 2, 3))
    got = paddle.nn.functional.affine_grid(paddle.to_tensor(theta), [2, 3, 5, 7], align_corners=True).numpy()
    np.testing.assert_allclose(got, affine_grid_np(theta, 2, 5, 7), rtol=1e-6, atol=1e-9)


@pytest.mark.parametrize("mode", ["bilinear", "nearest"])
@pytest.mark.parametrize("pad", ["zeros", "border", "reflection"])
@pytest.mark.parametrize("align", [True, False])
def test_grid_sample(mode, pad, align):
    data = R.uniform(-1, 1, (2, 3, 5, 6))
    grid = R.uniform(-1.3, 1.3, (2, 4, 7, 2))
    got = paddle.nn.functional.grid_sample(paddle.to_tensor(data), paddle.to_tensor(grid), mode=mode,
                                           padding_mode=pad, align_corners=align).numpy()
    np.testing.assert_allclose(got, grid_sample_np(data, grid, align, mode, pad), rtol=1e-5, atol=1e-7)
