"""avg/max pooling against the reference's naive numpy oracles
(python/paddle/fluid/tests/unittests/test_pool2d_op.py avg_pool2D_forward_naive /
max_pool2D_forward_naive, re-stated): exclusive vs inclusive divisor, ceil_mode, padding."""
import numpy as np
import pytest

import paddle_hackathon_amd as paddle

R = np.random.RandomState(5)


def pool_np(x, k, s, p, ceil_mode, exclusive, kind):
    N, C, H, W = x.shape
    if ceil_mode:
        Ho = (H - k[0] + 2 * p[0] + s[0] - 1) // s[0] + 1
        Wo = (W - k[1] + 2 * p[1] + s[1] - 1) // s[1] + 1
    else:
        Ho = (H - k[0] + 2 * p[0]) // s[0] + 1
        Wo = (W - k[1] + 2 * p[1]) // s[1] + 1
    out = np.zeros((N, C, Ho, Wo))
    for i in range(Ho):
        for j in range(Wo):
            r0, r1 = i * s[0] - p[0], i * s[0] + k[0] - p[0]
            c0, c1 = j * s[1] - p[1], j * s[1] + k[1] - p[1]
            field = (r1 - r0) * (c1 - c0)
            r0, r1, c0, c1 = max(r0, 0), min(r1, H), max(c0, 0), min(c1, W)
            xm = x[:, :, r0:r1, c0:c1]
            if kind == "max":
                out[:, :, i, j] = xm.max(axis=(2, 3))
            else:
                if exclusive:
                    field = (r1 - r0) * (c1 - c0)
                out[:, :, i, j] = xm.sum(axis=(2, 3)) / field
    return out


CASES = [  # (H, W, k, s, p) chosen so every ceil-mode window still overlaps the input
    (7, 7, (3, 3), (2, 2), (1, 1)),
    (8, 6, (2, 3), (2, 2), (0, 1)),
    (9, 9, (3, 3), (3, 3), (0, 0)),
    (6, 7, (3, 2), (2, 2), (1, 0)),
]


@pytest.mark.parametrize("H,W,k,s,p", CASES)
@pytest.mark.parametrize("ceil_mode", [False, True])
@pytest.mark.parametrize("exclusive", [True, False])
def test_avg_pool2d(H, W, k, s, p, ceil_mode, exclusive):
    x = R.uniform(-1, 1, (2, 3, H, W))
    got = paddle.nn.functional.avg_pool2d(paddle.to_tensor(x), list(k), list(s), list(p), ceil_mode=ceil_mode,
                                          exclusive=exclusive).numpy()
    np.testing.assert_allclose(got, pool_np(x, k, s, p, ceil_mode, exclusive, "avg"), rtol=1e-6, atol=1e-9)


@pytest.mark.parametrize("H,W,k,s,p", CASES)
@pytest.mark.parametrize("ceil_mode", [False, True])
def test_max_pool2d(H, W, k, s, p, ceil_mode):
    x = R.uniform(-1, 1, (2, 3, H, W))
    got = paddle.nn.functional.max_pool2d(paddle.to_tensor(x), list(k), list(s), list(p),
                                          ceil_mode=ceil_mode).numpy()
    np.testing.assert_allclose(got, pool_np(x, k, s, p, ceil_mode, True, "max"))


def test_avg_pool1d_inclusive_ceil():
    x = R.uniform(-1, 1, (2, 3, 8))
    got = paddle.nn.functional.avg_pool1d(paddle.to_tensor(x), 3, 3, 1, exclusive=False, ceil_mode=True).numpy()
    want = pool_np(x[:, :, None, :], (1, 3), (1, 3), (0, 1), True, False, "avg")[:, :, 0, :]
    np.testing.assert_allclose(got, want, rtol=1e-6, atol=1e-9)


def test_ceil_mode_keeps_window_starting_in_padding():
    """reference output size: a last window that starts in the padding is kept (shape parity)"""
    x = R.uniform(-1, 1, (1, 2, 8, 8))
    for fn, kw in ((paddle.nn.functional.max_pool2d, {}), (paddle.nn.functional.avg_pool2d, {"exclusive": False})):
        got = fn(paddle.to_tensor(x), 3, 3, 1, ceil_mode=True, **kw).numpy()
        assert got.shape == (1, 2, 4, 4)
        # the windows that overlap the input are the non-ceil ones; the kept tail window is empty
        np.testing.assert_allclose(got[:, :, :3, :3], pool_np(x, (3, 3), (3, 3), (1, 1), False, False,
                                                             "max" if not kw else "avg"))
        tail = got[:, :, 3, :]
        assert (tail == (np.finfo(got.dtype).min if not kw else 0.0)).all()
