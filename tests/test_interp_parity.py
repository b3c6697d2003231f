"""nn.functional.interpolate against the reference's numpy oracles
(python/paddle/fluid/tests/unittests/test_{bilinear,nearest,linear}_interp_v2_op.py, re-stated):
align_corners, align_mode 0 (half pixel) and 1 (asymmetric), scale vs size."""
import numpy as np
import pytest

import paddle_hackathon_amd as paddle

R = np.random.RandomState(11)


def _ratio(n_in, n_out, align_corners, scale):
    if n_out <= 1:
        return 0.0
    if align_corners:
        return (n_in - 1.0) / (n_out - 1.0)
    return 1.0 / scale if scale > 0 else 1.0 * n_in / n_out


def bilinear_np(x, out_h, out_w, align_corners, align_mode, scale_h=0, scale_w=0):
    n, c, in_h, in_w = x.shape
    rh, rw = _ratio(in_h, out_h, align_corners, scale_h), _ratio(in_w, out_w, align_corners, scale_w)
    half = align_mode == 0 and not align_corners
    out = np.zeros((n, c, out_h, out_w))
    for i in range(out_h):
        h = max(0, int(rh * (i + 0.5) - 0.5) if half else int(rh * i))
        hid = 1 if h < in_h - 1 else 0
        l1 = (max(rh * (i + 0.5) - 0.5, 0) - h) if half else rh * i - h
        for j in range(out_w):
            w = max(0, int(rw * (j + 0.5) - 0.5) if half else int(rw * j))
            wid = 1 if w < in_w - 1 else 0
            m1 = (max(rw * (j + 0.5) - 0.5, 0) - w) if half else rw * j - w
            out[:, :, i, j] = (1 - l1) * ((1 - m1) * x[:, :, h, w] + m1 * x[:, :, h, w + wid]) + \
                l1 * ((1 - m1) * x[:, :, h + hid, w] + m1 * x[:, :, h + hid, w + wid])
    return out


def nearest_np(x, out_h, out_w, align_corners):
    n, c, in_h, in_w = x.shape
    rh, rw = _ratio(in_h, out_h, align_corners, 0), _ratio(in_w, out_w, align_corners, 0)
    out = np.zeros((n, c, out_h, out_w))
    for i in range(out_h):
        ii = int(rh * i + 0.5) if align_corners else int(rh * i)
        for j in range(out_w):
            jj = int(rw * j + 0.5) if align_corners else int(rw * j)
            out[:, :, i, j] = x[:, :, ii, jj]
    return out


@pytest.mark.parametrize("align_corners,align_mode", [(True, 0), (False, 0), (False, 1)])
@pytest.mark.parametrize("out_hw", [(9, 12), (3, 5), (4, 4)])
def test_bilinear(align_corners, align_mode, out_hw):
    x = R.uniform(-1, 1, (2, 3, 5, 7))
    got = paddle.nn.functional.interpolate(paddle.to_tensor(x), size=list(out_hw), mode="bilinear",
                                           align_corners=align_corners, align_mode=align_mode).numpy()
    np.testing.assert_allclose(got, bilinear_np(x, *out_hw, align_corners, align_mode), rtol=1e-6, atol=1e-9)


def test_bilinear_scale_factor_align_mode1():
    x = R.uniform(-1, 1, (1, 2, 4, 6))
    got = paddle.nn.functional.interpolate(paddle.to_tensor(x), scale_factor=[1.5, 2.0], mode="bilinear",
                                           align_corners=False, align_mode=1).numpy()
    np.testing.assert_allclose(got, bilinear_np(x, 6, 12, False, 1, 1.5, 2.0), rtol=1e-6, atol=1e-9)


@pytest.mark.parametrize("align_corners", [True, False])
@pytest.mark.parametrize("out_hw", [(9, 12), (3, 5)])
def test_nearest(align_corners, out_hw):
    x = R.uniform(-1, 1, (2, 3, 5, 7))
    got = paddle.nn.functional.interpolate(paddle.to_tensor(x), size=list(out_hw), mode="nearest",
                                           align_corners=align_corners).numpy()
    np.testing.assert_allclose(got, nearest_np(x, *out_hw, align_corners))


def test_linear_nlc():
    x = R.uniform(-1, 1, (2, 7, 3))          # NLC
    got = paddle.nn.functional.interpolate(paddle.to_tensor(x), size=[11], mode="linear", align_corners=False,
                                           align_mode=1, data_format="NLC").numpy()
    ref = bilinear_np(x.transpose(0, 2, 1)[:, :, None, :], 1, 11, False, 1)[:, :, 0, :].transpose(0, 2, 1)
    np.testing.assert_allclose(got, ref, rtol=1e-6, atol=1e-9)
