"""Op-semantics parity against the reference's own numpy oracles (no torch in the oracle).

Each case re-states the numpy computation the reference's OpTest / API test uses for the op
(python/paddle/fluid/tests/unittests/test_<op>_op.py: ``self.outputs = {...}`` built with numpy, or
the ``ref_*`` / ``*_np`` helpers), runs our ``paddle.*`` API on the same inputs and compares.
The file that holds the oracle is named per case (``src``). Cases where the reference kernel and
its fixture disagree on an input class the fixture never exercises (e.g. ``round`` at exact .5:
kernel uses std::round, fixture np.round on uniform(-1, 1)) are tested on the fixture's input class
and noted.
"""
import math

import numpy as np
import pytest

import paddle_hackathon_amd as paddle

pytestmark = pytest.mark.timeout(300)

R = np.random.RandomState(2022)


def U(*shape, lo=-1.0, hi=1.0, dtype="float64"):
    return R.uniform(lo, hi, shape).astype(dtype)


def P(x):
    return paddle.to_tensor(x)


def _erf(x):
    return np.vectorize(math.erf)(x)


def _gamma_ln(x):
    return np.vectorize(math.lgamma)(x)


def softmax_np(x, axis=-1):
    e = np.exp(x - x.max(axis=axis, keepdims=True))
    return e / e.sum(axis=axis, keepdims=True)


# ----------------------------------------------------------------------------- unary / activation
x_a = U(4, 7, lo=-3, hi=3)
x_pos = U(4, 7, lo=0.1, hi=4)
x_unit = U(4, 7, lo=-0.95, hi=0.95)
x_gt1 = U(4, 7, lo=1.05, hi=4)

UNARY = [
    # (name, api, numpy oracle, input, source)
    ("abs", paddle.abs, np.abs, x_a, "test_activation_op.py TestAbs"),
    ("exp", paddle.exp, np.exp, x_a, "test_activation_op.py TestExp"),
    ("expm1", paddle.expm1, np.expm1, x_a, "test_activation_op.py TestExpm1"),
    ("log", paddle.log, np.log, x_pos, "test_activation_op.py TestLog"),
    ("log2", paddle.log2, np.log2, x_pos, "test_activation_op.py TestLog2"),
    ("log10", paddle.log10, np.log10, x_pos, "test_activation_op.py TestLog10"),
    ("log1p", paddle.log1p, np.log1p, x_pos, "test_activation_op.py TestLog1p"),
    ("sqrt", paddle.sqrt, np.sqrt, x_pos, "test_activation_op.py TestSqrt"),
    ("rsqrt", paddle.rsqrt, lambda x: 1.0 / np.sqrt(x), x_pos, "test_activation_op.py TestRsqrt"),
    ("square", paddle.square, np.square, x_a, "test_activation_op.py TestSquare"),
    ("reciprocal", paddle.reciprocal, np.reciprocal, x_pos, "test_activation_op.py TestReciprocal"),
    ("sign", paddle.sign, np.sign, x_a, "test_sign_op.py"),
    ("floor", paddle.floor, np.floor, x_a, "test_activation_op.py TestFloor"),
    ("ceil", paddle.ceil, np.ceil, x_a, "test_activation_op.py TestCeil"),
    ("round", paddle.round, np.round, x_unit, "test_activation_op.py TestRound (uniform(-1,1), no exact .5)"),
    ("trunc", paddle.trunc, np.trunc, x_a, "test_trunc_op.py"),
    ("sin", paddle.sin, np.sin, x_a, "test_activation_op.py TestSin"),
    ("cos", paddle.cos, np.cos, x_a, "test_activation_op.py TestCos"),
    ("tan", paddle.tan, np.tan, x_unit, "test_activation_op.py TestTan"),
    ("asin", paddle.asin, np.arcsin, x_unit, "test_activation_op.py TestAsin"),
    ("acos", paddle.acos, np.arccos, x_unit, "test_activation_op.py TestAcos"),
    ("atan", paddle.atan, np.arctan, x_a, "test_activation_op.py TestAtan"),
    ("sinh", paddle.sinh, np.sinh, x_a, "test_activation_op.py TestSinh"),
    ("cosh", paddle.cosh, np.cosh, x_a, "test_activation_op.py TestCosh"),
    ("tanh", paddle.tanh, np.tanh, x_a, "test_activation_op.py TestTanh"),
    ("asinh", paddle.asinh, np.arcsinh, x_a, "test_activation_op.py TestAsinh"),
    ("acosh", paddle.acosh, np.arccosh, x_gt1, "test_activation_op.py TestAcosh"),
    ("atanh", paddle.atanh, np.arctanh, x_unit, "test_activation_op.py TestAtanh"),
    ("erf", paddle.erf, _erf, x_a, "test_erf_op.py (scipy.special.erf)"),
    ("lgamma", paddle.lgamma, _gamma_ln, x_pos, "test_lgamma_op.py (math.lgamma)"),
    ("sigmoid", paddle.nn.functional.sigmoid, lambda x: 1 / (1 + np.exp(-x)), x_a, "test_activation_op.py TestSigmoid"),
    ("logsigmoid", paddle.nn.functional.log_sigmoid, lambda x: np.log(1 / (1 + np.exp(-x))), x_a,
     "test_activation_op.py TestLogSigmoid"),
    ("relu", paddle.nn.functional.relu, lambda x: np.maximum(x, 0), x_a, "test_activation_op.py TestRelu"),
    ("relu6", paddle.nn.functional.relu6, lambda x: np.minimum(np.maximum(x, 0), 6.0), U(4, 7, lo=-10, hi=10),
     "test_activation_op.py ref_relu6"),
    ("leaky_relu", lambda x: paddle.nn.functional.leaky_relu(x, 0.02), lambda x: np.where(x > 0, x, 0.02 * x), x_a,
     "test_activation_op.py ref_leaky_relu"),
    ("elu", lambda x: paddle.nn.functional.elu(x, 0.7), lambda x: np.where(x > 0, x, 0.7 * (np.exp(x) - 1)), x_a,
     "test_activation_op.py elu"),
    ("celu", lambda x: paddle.nn.functional.celu(x, 1.5),
     lambda x: np.maximum(0, x) + np.minimum(0, 1.5 * (np.exp(x / 1.5) - 1)), x_a, "test_activation_op.py ref_celu"),
    ("selu", paddle.nn.functional.selu,
     lambda x: 1.0507009873554804934193349852946 * np.where(x > 0, x, 1.6732632423543772848170429916717 * (np.exp(x) - 1)),
     x_a, "test_selu_op.py ref_selu"),
    ("gelu", paddle.nn.functional.gelu, lambda x: 0.5 * x * (1 + _erf(x / np.sqrt(2))), x_a,
     "test_gelu_op.py gelu(approximate=False)"),
    ("gelu_tanh", lambda x: paddle.nn.functional.gelu(x, approximate=True),
     lambda x: 0.5 * x * (1 + np.tanh(np.sqrt(2 / np.pi) * (x + 0.044715 * x ** 3))), x_a,
     "test_gelu_op.py gelu(approximate=True)"),
    ("silu", paddle.nn.functional.silu, lambda x: x / (1 + np.exp(-x)), x_a, "test_activation_op.py TestSilu"),
    ("swish", paddle.nn.functional.swish, lambda x: x / (1 + np.exp(-x)), x_a, "test_activation_op.py ref_swish"),
    ("hardswish", paddle.nn.functional.hardswish, lambda x: x * np.minimum(np.maximum(x + 3, 0), 6) / 6,
     U(4, 7, lo=-6, hi=6), "test_activation_op.py ref_hardswish"),
    ("hardsigmoid", paddle.nn.functional.hardsigmoid,
     lambda x: np.maximum(np.minimum(x * 0.166666666666667 + 0.5, 1), 0), U(4, 7, lo=-5, hi=5),
     "test_activation_op.py ref_hardsigmoid"),
    ("hardtanh", paddle.nn.functional.hardtanh, lambda x: np.clip(x, -1, 1), x_a, "test_activation_op.py ref_hardtanh"),
    ("hardshrink", lambda x: paddle.nn.functional.hardshrink(x, 0.5), lambda x: np.where(np.abs(x) > 0.5, x, 0), x_a,
     "test_activation_op.py ref_hardshrink"),
    ("softshrink", lambda x: paddle.nn.functional.softshrink(x, 0.5),
     lambda x: np.where(x > 0.5, x - 0.5, np.where(x < -0.5, x + 0.5, 0)), x_a, "test_activation_op.py ref_softshrink"),
    ("tanhshrink", paddle.nn.functional.tanhshrink, lambda x: x - np.tanh(x), x_a, "test_activation_op.py ref_tanhshrink"),
    ("softsign", paddle.nn.functional.softsign, lambda x: x / (1 + np.abs(x)), x_a, "test_activation_op.py ref_softsign"),
    ("softplus", lambda x: paddle.nn.functional.softplus(x, beta=2, threshold=3),
     lambda x: np.where(2 * x <= 3, np.log(1 + np.exp(2 * x)) / 2, x), x_a, "test_activation_op.py ref_softplus"),
    ("mish", paddle.nn.functional.mish, lambda x: x * np.tanh(np.where(x <= 20, np.log(1 + np.exp(x)), x)), x_a,
     "test_activation_op.py ref_mish"),
    ("thresholded_relu", lambda x: paddle.nn.functional.thresholded_relu(x, 1.0), lambda x: np.where(x > 1.0, x, 0),
     x_a, "test_activation_op.py ref_thresholded_relu"),
    ("stanh", lambda x: paddle.stanh(x, 0.67, 1.7159), lambda x: 1.7159 * np.tanh(0.67 * x), x_a,
     "test_activation_op.py ref_stanh"),
    ("softmax", paddle.nn.functional.softmax, softmax_np, x_a, "test_softmax_op.py stable_softmax"),
    ("log_softmax", paddle.nn.functional.log_softmax, lambda x: np.log(softmax_np(x)), x_a,
     "test_log_softmax.py ref_log_softmax"),
    ("softmax_axis0", lambda x: paddle.nn.functional.softmax(x, axis=0), lambda x: softmax_np(x, 0), x_a,
     "test_softmax_op.py axis"),
    ("logit", lambda x: paddle.logit(x, 1e-3),
     lambda x: np.log(np.clip(x, 1e-3, 1 - 1e-3) / (1 - np.clip(x, 1e-3, 1 - 1e-3))), U(4, 7, lo=0, hi=1),
     "test_logit_op.py logit"),
    ("neg", paddle.neg, np.negative, x_a, "test_activation_op.py"),
    ("digamma", paddle.digamma, None, x_pos, "test_digamma_op.py (scipy.special.psi; checked by recurrence)"),
]


@pytest.mark.parametrize("name,api,ref,x,src", UNARY, ids=[u[0] for u in UNARY])
def test_unary(name, api, ref, x, src):
    got = api(P(x)).numpy()
    if name == "digamma":   # psi(x+1) - psi(x) = 1/x  (no scipy needed)
        got1 = api(P(x + 1)).numpy()
        np.testing.assert_allclose(got1 - got, 1.0 / x, rtol=1e-6, atol=1e-8)
        return
    np.testing.assert_allclose(got, ref(x), rtol=1e-6, atol=1e-7, err_msg=src)


# ----------------------------------------------------------------------------- binary elementwise
a_f, b_f = U(3, 4, 5, lo=-5, hi=5), U(3, 4, 5, lo=-5, hi=5)
b_nz = np.where(np.abs(b_f) < 0.5, 1.5, b_f)
a_i = R.randint(-20, 20, (3, 4, 5)).astype("int64")
b_i = R.randint(-7, 7, (3, 4, 5)).astype("int64")
b_i[b_i == 0] = 3

BINARY = [
    ("add", paddle.add, np.add, a_f, b_f, "test_elementwise_add_op.py"),
    ("subtract", paddle.subtract, np.subtract, a_f, b_f, "test_elementwise_sub_op.py"),
    ("multiply", paddle.multiply, np.multiply, a_f, b_f, "test_elementwise_mul_op.py"),
    ("divide", paddle.divide, np.divide, a_f, b_nz, "test_elementwise_div_op.py"),
    ("pow", paddle.pow, np.power, np.abs(a_f) + 0.1, b_f / 3, "test_elementwise_pow_op.py"),
    ("maximum", paddle.maximum, np.maximum, a_f, b_f, "test_elementwise_max_op.py"),
    ("minimum", paddle.minimum, np.minimum, a_f, b_f, "test_elementwise_min_op.py"),
    ("fmax", paddle.fmax, np.fmax, a_f, b_f, "test_fmax_op.py"),
    ("fmin", paddle.fmin, np.fmin, a_f, b_f, "test_fmin_op.py"),
    # reference floor_divide kernel truncates toward zero (elementwise_functor.h:555-561)
    ("floor_divide_int", paddle.floor_divide, lambda a, b: np.trunc(a / b).astype("int64"), a_i, b_i,
     "test_elementwise_floordiv_op.py + kernel trunc"),
    ("remainder_int", paddle.remainder, np.mod, a_i, b_i, "test_elementwise_mod_op.py (np.mod: sign of divisor)"),
    ("remainder_float", paddle.remainder, np.fmod, np.abs(a_f), np.abs(b_nz), "test_elementwise_mod_op.py float"),
    ("atan2", paddle.atan2, np.arctan2, a_f, b_f, "test_atan2_op.py"),
    ("broadcast_add", paddle.add, np.add, a_f, U(5), "test_elementwise_add_op.py broadcast"),
    ("broadcast_mul_mid", paddle.multiply, np.multiply, a_f, U(4, 1), "test_elementwise_mul_op.py broadcast"),
    ("heaviside", paddle.heaviside, np.heaviside, a_f, b_f, "test_elementwise_heaviside_op.py"),
]


@pytest.mark.parametrize("name,api,ref,a,b,src", BINARY, ids=[u[0] for u in BINARY])
def test_binary(name, api, ref, a, b, src):
    got = api(P(a), P(b)).numpy()
    np.testing.assert_allclose(got, ref(a, b), rtol=1e-6, atol=1e-7, err_msg=src)


COMPARE = [
    ("equal", paddle.equal, np.equal), ("not_equal", paddle.not_equal, np.not_equal),
    ("less_than", paddle.less_than, np.less), ("less_equal", paddle.less_equal, np.less_equal),
    ("greater_than", paddle.greater_than, np.greater), ("greater_equal", paddle.greater_equal, np.greater_equal),
    ("logical_and", paddle.logical_and, np.logical_and), ("logical_or", paddle.logical_or, np.logical_or),
    ("logical_xor", paddle.logical_xor, np.logical_xor),
    ("bitwise_and", paddle.bitwise_and, np.bitwise_and), ("bitwise_or", paddle.bitwise_or, np.bitwise_or),
    ("bitwise_xor", paddle.bitwise_xor, np.bitwise_xor),
]


@pytest.mark.parametrize("name,api,ref", COMPARE, ids=[c[0] for c in COMPARE])
def test_compare_logic(name, api, ref):
    a = R.randint(-3, 3, (4, 6)).astype("int64")
    b = R.randint(-3, 3, (4, 6)).astype("int64")
    if name.startswith("logical"):
        a, b = a > 0, b > 0
    np.testing.assert_array_equal(api(P(a), P(b)).numpy(), ref(a, b), err_msg=f"test_compare_op.py / test_logical_op.py {name}")


def test_round_half_away_from_zero():
    # kernel: Eigen x.round() == std::round (activation_functor.h RoundFunctor); the fixture never hits .5
    x = np.array([0.5, 1.5, 2.5, -0.5, -2.5, 0.49999997, 3.2, -3.7])
    want = np.sign(x) * np.floor(np.abs(x) + 0.5)
    want[5] = 0.0
    np.testing.assert_array_equal(paddle.round(P(x)).numpy(), want)
    t = P(x.copy())
    t.round_()
    np.testing.assert_array_equal(t.numpy(), want)


def test_unary_logic():
    a = R.randint(-3, 3, (4, 6)).astype("int64")
    np.testing.assert_array_equal(paddle.bitwise_not(P(a)).numpy(), np.invert(a))
    np.testing.assert_array_equal(paddle.logical_not(P(a > 0)).numpy(), a <= 0)
    x = np.array([1.0, np.nan, np.inf, -np.inf, 0.0])
    np.testing.assert_array_equal(paddle.isnan(P(x)).numpy(), np.isnan(x))
    np.testing.assert_array_equal(paddle.isinf(P(x)).numpy(), np.isinf(x))
    np.testing.assert_array_equal(paddle.isfinite(P(x)).numpy(), np.isfinite(x))
    y = x + 1e-9
    np.testing.assert_array_equal(paddle.isclose(P(x), P(y), equal_nan=True).numpy(),
                                  np.isclose(x, y, equal_nan=True))


# ----------------------------------------------------------------------------- reductions / stats
xr = U(3, 4, 5, lo=-2, hi=2)

REDUCE = [
    ("sum_all", lambda t: paddle.sum(t), lambda x: np.sum(x), "test_reduce_op.py TestSumOp"),
    ("sum_axis", lambda t: paddle.sum(t, axis=1), lambda x: x.sum(1), "test_reduce_op.py"),
    ("sum_axes_keep", lambda t: paddle.sum(t, axis=[0, 2], keepdim=True), lambda x: x.sum((0, 2), keepdims=True),
     "test_reduce_op.py keep_dim"),
    ("mean", lambda t: paddle.mean(t, axis=-1), lambda x: x.mean(-1), "test_mean_op.py"),
    ("max", lambda t: paddle.max(t, axis=0), lambda x: x.max(0), "test_reduce_op.py TestMaxOp"),
    ("min", lambda t: paddle.min(t, axis=2), lambda x: x.min(2), "test_reduce_op.py TestMinOp"),
    ("prod", lambda t: paddle.prod(t, axis=1), lambda x: x.prod(1), "test_reduce_op.py TestProdOp"),
    ("logsumexp", lambda t: paddle.logsumexp(t, axis=1), lambda x: np.log(np.exp(x).sum(1)), "test_logsumexp.py"),
    ("var", lambda t: paddle.var(t, axis=1), lambda x: x.var(1, ddof=1), "test_variance_layer.py (unbiased)"),
    ("std_biased", lambda t: paddle.std(t, axis=2, unbiased=False), lambda x: x.std(2), "test_std_layer.py"),
    # reference median averages the two middle values for even counts (test_median.py np.median)
    ("median_even", lambda t: paddle.median(t, axis=1), lambda x: np.median(x, 1), "test_median.py"),
    ("median_all", lambda t: paddle.median(t), lambda x: np.median(x), "test_median.py"),
    ("nanmean", lambda t: paddle.nanmean(t, axis=0), lambda x: np.nanmean(x, 0), "test_nanmean_api.py"),
    ("amax", lambda t: paddle.amax(t, axis=1), lambda x: x.max(1), "test_max_min_amax_amin_op.py"),
    ("cumsum", lambda t: paddle.cumsum(t, axis=1), lambda x: np.cumsum(x, 1), "test_cumsum_op.py"),
    ("cumsum_flat", lambda t: paddle.cumsum(t), lambda x: np.cumsum(x.reshape(-1)), "test_cumsum_op.py axis=None"),
    ("cumprod", lambda t: paddle.cumprod(t, dim=2), lambda x: np.cumprod(x, 2), "test_cumprod_op.py"),
    ("argmax", lambda t: paddle.argmax(t, axis=1), lambda x: x.argmax(1), "test_arg_min_max_op.py"),
    ("argmin", lambda t: paddle.argmin(t, axis=-1), lambda x: x.argmin(-1), "test_arg_min_max_op.py"),
    ("argmax_flat", lambda t: paddle.argmax(t), lambda x: np.array(x.argmax()), "test_arg_min_max_op.py axis=None"),
    ("norm_fro", lambda t: paddle.linalg.norm(t), lambda x: np.sqrt((x ** 2).sum()), "test_norm_all.py frobenius"),
    ("norm_p3", lambda t: paddle.linalg.norm(t, p=3, axis=1), lambda x: (np.abs(x) ** 3).sum(1) ** (1 / 3),
     "test_norm_all.py p_norm"),
    ("norm_inf", lambda t: paddle.linalg.norm(t, p=np.inf, axis=2), lambda x: np.abs(x).max(2), "test_norm_all.py inf"),
    ("count_nonzero", lambda t: paddle.count_nonzero(t > 0, axis=1), lambda x: (x > 0).sum(1), "test_count_nonzero_api.py"),
    ("all", lambda t: paddle.all(t > -1.9, axis=1), lambda x: (x > -1.9).all(1), "test_reduce_op.py TestAllOp"),
    ("any", lambda t: paddle.any(t > 1.9, axis=1), lambda x: (x > 1.9).any(1), "test_reduce_op.py TestAnyOp"),
]


@pytest.mark.parametrize("name,api,ref,src", REDUCE, ids=[c[0] for c in REDUCE])
def test_reduce(name, api, ref, src):
    got = api(P(xr)).numpy()
    want = np.asarray(ref(xr))
    np.testing.assert_allclose(got.reshape(want.shape) if got.size == want.size else got, want, rtol=1e-6, atol=1e-7,
                               err_msg=src)


def test_full_reductions_have_shape_one():
    # the reference has no 0-d tensors: full reductions are shape [1] (``loss.numpy()[0]``)
    t = P(xr)
    for r in (paddle.sum(t), paddle.mean(t), paddle.max(t), t.sum()):
        assert r.shape == [1]
        assert r.numpy().shape == (1,)
        r.numpy()[0]


def test_topk_sort_kthvalue_mode():
    x = U(4, 9)
    v, i = paddle.topk(P(x), 3, axis=1)
    idx = np.argsort(-x, axis=1)[:, :3]
    np.testing.assert_allclose(v.numpy(), np.take_along_axis(x, idx, 1))
    np.testing.assert_array_equal(i.numpy(), idx)
    v, i = paddle.topk(P(x), 2, axis=1, largest=False)
    np.testing.assert_allclose(v.numpy(), np.sort(x, 1)[:, :2])
    np.testing.assert_allclose(paddle.sort(P(x), axis=1, descending=True).numpy(), -np.sort(-x, 1))
    np.testing.assert_array_equal(paddle.argsort(P(x), axis=0).numpy(), np.argsort(x, 0, kind="stable"))
    v, i = paddle.kthvalue(P(x), 4, axis=1)
    np.testing.assert_allclose(v.numpy(), np.sort(x, 1)[:, 3])
    xi = np.array([[1, 2, 2, 3, 3, 3], [5, 5, 4, 4, 4, 1]], dtype="int64")
    v, i = paddle.mode(P(xi), axis=1)
    np.testing.assert_array_equal(v.numpy(), [3, 4])


# ----------------------------------------------------------------------------- manipulation
def test_manipulation():
    x = U(2, 3, 4)
    np.testing.assert_allclose(paddle.concat([P(x), P(x)], axis=1).numpy(), np.concatenate([x, x], 1))
    np.testing.assert_allclose(paddle.stack([P(x), P(x)], axis=2).numpy(), np.stack([x, x], 2))
    parts = paddle.split(P(x), [1, -1], axis=2)
    np.testing.assert_allclose(parts[1].numpy(), x[:, :, 1:])
    parts = paddle.split(P(x), 2, axis=0)
    np.testing.assert_allclose(parts[1].numpy(), x[1:])
    np.testing.assert_allclose(paddle.reshape(P(x), [0, -1]).numpy(), x.reshape(2, -1))   # 0 copies the dim
    np.testing.assert_allclose(paddle.transpose(P(x), [2, 0, 1]).numpy(), x.transpose(2, 0, 1))
    np.testing.assert_allclose(paddle.flatten(P(x), 1, 2).numpy(), x.reshape(2, 12))
    np.testing.assert_allclose(paddle.unsqueeze(P(x), [0, 2]).numpy(), x[None, :, None])
    np.testing.assert_allclose(paddle.squeeze(P(x[:, :1]), axis=1).numpy(), x[:, 0])
    np.testing.assert_allclose(paddle.tile(P(x), [2, 1, 1]).numpy(), np.tile(x, (2, 1, 1)))
    np.testing.assert_allclose(paddle.expand(P(x[:, :1]), [2, 3, 4]).numpy(), np.broadcast_to(x[:, :1], (2, 3, 4)))
    np.testing.assert_allclose(paddle.flip(P(x), [0, 2]).numpy(), x[::-1, :, ::-1])
    np.testing.assert_allclose(paddle.roll(P(x), 2, axis=2).numpy(), np.roll(x, 2, 2))
    np.testing.assert_allclose(paddle.roll(P(x), 3).numpy(), np.roll(x, 3))
    idx = np.array([2, 0])
    np.testing.assert_allclose(paddle.gather(P(x), P(idx), axis=1).numpy(), x[:, idx])
    nd = np.array([[0, 1], [1, 2]])
    np.testing.assert_allclose(paddle.gather_nd(P(x), P(nd)).numpy(), x[nd[:, 0], nd[:, 1]])
    np.testing.assert_allclose(paddle.index_select(P(x), P(idx), axis=2).numpy(), x[:, :, idx])
    m = x > 0
    np.testing.assert_allclose(paddle.masked_select(P(x), P(m)).numpy(), x[m])
    np.testing.assert_allclose(paddle.where(P(m), P(x), P(-x)).numpy(), np.where(m, x, -x))
    np.testing.assert_allclose(paddle.tril(P(x[0]), 1).numpy(), np.tril(x[0], 1))
    np.testing.assert_allclose(paddle.triu(P(x[0]), -1).numpy(), np.triu(x[0], -1))
    np.testing.assert_allclose(paddle.diag(P(x[0, 0])).numpy(), np.diag(x[0, 0]))
    np.testing.assert_allclose(paddle.diagonal(P(x), 0, 1, 2).numpy(), np.diagonal(x, 0, 1, 2))
    ids = np.array([[1], [3], [0]])
    np.testing.assert_allclose(paddle.take_along_axis(P(x[0]), P(ids), 1).numpy(), np.take_along_axis(x[0], ids, 1))
    np.testing.assert_allclose(paddle.repeat_interleave(P(x), 2, axis=1).numpy(), np.repeat(x, 2, 1))
    np.testing.assert_array_equal(paddle.nonzero(P(m)).numpy(), np.stack(np.nonzero(m), 1))
    u, inv, cnt = paddle.unique(P(np.array([3, 1, 3, 2, 1])), return_inverse=True, return_counts=True)
    nu, ninv, ncnt = np.unique(np.array([3, 1, 3, 2, 1]), return_inverse=True, return_counts=True)
    np.testing.assert_array_equal(u.numpy(), nu)
    np.testing.assert_array_equal(inv.numpy(), ninv)
    np.testing.assert_array_equal(cnt.numpy(), ncnt)
    oh = paddle.nn.functional.one_hot(P(np.array([0, 2, 1])), 4).numpy()
    np.testing.assert_array_equal(oh, np.eye(4)[[0, 2, 1]])
    g = paddle.meshgrid(P(np.arange(3.0)), P(np.arange(2.0)))
    ng = np.meshgrid(np.arange(3.0), np.arange(2.0), indexing="ij")
    np.testing.assert_allclose(g[0].numpy(), ng[0])
    np.testing.assert_allclose(paddle.strided_slice(P(x), [1, 2], [0, 3], [3, 0], [2, -1]).numpy(), x[:, 0:3:2, 3:0:-1])
    np.testing.assert_allclose(paddle.slice(P(x), [0, 2], [1, 1], [2, 3]).numpy(), x[1:2, :, 1:3])
    np.testing.assert_allclose(paddle.chunk(P(x), 2, axis=2)[1].numpy(), x[:, :, 2:])
    np.testing.assert_allclose(paddle.unbind(P(x), 1)[2].numpy(), x[:, 2])
    np.testing.assert_allclose(paddle.broadcast_to(P(x[:1]), [2, 3, 4]).numpy(), np.broadcast_to(x[:1], (2, 3, 4)))


def test_scatter_family():
    x = U(5, 3)
    idx = np.array([1, 3, 1])
    upd = U(3, 3)
    # overwrite=True: the last update of a repeated index wins (test_scatter_op.py)
    ref = x.copy()
    for k, i in enumerate(idx):
        ref[i] = upd[k]
    np.testing.assert_allclose(paddle.scatter(P(x), P(idx), P(upd)).numpy(), ref)
    # overwrite=False: repeated rows are zeroed then summed (test_scatter_op.py TestScatterOp0 overwrite False)
    ref = x.copy()
    for i in idx:
        ref[i] = 0
    for k, i in enumerate(idx):
        ref[i] += upd[k]
    np.testing.assert_allclose(paddle.scatter(P(x), P(idx), P(upd), overwrite=False).numpy(), ref)
    nd = np.array([[1], [3], [1]])
    ref = x.copy()
    for k, i in enumerate(nd[:, 0]):
        ref[i] += upd[k]
    np.testing.assert_allclose(paddle.scatter_nd_add(P(x), P(nd), P(upd)).numpy(), ref)
    ref = x.copy()
    np.put_along_axis(ref, np.array([[0], [2], [1], [0], [2]]), 9.0, 1)
    np.testing.assert_allclose(paddle.put_along_axis(P(x), P(np.array([[0], [2], [1], [0], [2]])), 9.0, 1).numpy(), ref)


# ----------------------------------------------------------------------------- creation / search
def test_creation_search():
    np.testing.assert_allclose(paddle.arange(1, 10, 2.5).numpy(), np.arange(1, 10, 2.5))
    np.testing.assert_allclose(paddle.linspace(0, 1, 7).numpy(), np.linspace(0, 1, 7), rtol=1e-6)
    np.testing.assert_allclose(paddle.logspace(0, 2, 5, base=10).numpy(), np.logspace(0, 2, 5), rtol=1e-5)
    np.testing.assert_allclose(paddle.eye(3, 4).numpy(), np.eye(3, 4))
    np.testing.assert_allclose(paddle.full([2, 3], 1.5).numpy(), np.full((2, 3), 1.5))
    s = np.array([1.0, 3.0, 5.0, 7.0])
    v = np.array([0.5, 3.0, 6.0, 9.0])
    np.testing.assert_array_equal(paddle.searchsorted(P(s), P(v)).numpy(), np.searchsorted(s, v))
    np.testing.assert_array_equal(paddle.searchsorted(P(s), P(v), right=True).numpy(), np.searchsorted(s, v, "right"))
    h = R.uniform(0, 4, 50)
    np.testing.assert_array_equal(paddle.histogram(P(h), bins=4, min=0, max=4).numpy(),
                                  np.histogram(h, 4, (0, 4))[0])
    b = np.array([0, 1, 1, 3, 3, 3])
    np.testing.assert_array_equal(paddle.bincount(P(b)).numpy(), np.bincount(b))


# ----------------------------------------------------------------------------- linalg
def test_linalg():
    a, b = U(3, 4, 5), U(3, 5, 2)
    np.testing.assert_allclose(paddle.matmul(P(a), P(b)).numpy(), a @ b, rtol=1e-10)
    np.testing.assert_allclose(paddle.matmul(P(a), P(a), transpose_y=True).numpy(), a @ a.transpose(0, 2, 1))
    np.testing.assert_allclose(paddle.bmm(P(a), P(b)).numpy(), a @ b)
    v = U(5)
    np.testing.assert_allclose(paddle.matmul(P(a), P(v)).numpy(), a @ v)   # 1-D y squeezes
    np.testing.assert_allclose(paddle.dot(P(v), P(v)).numpy().reshape(-1), [v @ v])
    np.testing.assert_allclose(paddle.mv(P(a[0]), P(v)).numpy(), a[0] @ v)
    c1, c2 = U(4, 3), U(4, 3)
    np.testing.assert_allclose(paddle.cross(P(c1), P(c2), axis=1).numpy(), np.cross(c1, c2, axis=1))
    np.testing.assert_allclose(paddle.dist(P(c1), P(c2), p=2).numpy().reshape(-1), [np.linalg.norm(c1 - c2)])
    m = U(4, 4) + 4 * np.eye(4)
    spd = m @ m.T
    np.testing.assert_allclose(paddle.linalg.cholesky(P(spd)).numpy(), np.linalg.cholesky(spd), rtol=1e-8)
    np.testing.assert_allclose(paddle.linalg.inv(P(m)).numpy(), np.linalg.inv(m), rtol=1e-8)
    np.testing.assert_allclose(paddle.linalg.det(P(m)).numpy().reshape(-1), [np.linalg.det(m)], rtol=1e-8)
    sgn, logdet = np.linalg.slogdet(m)
    np.testing.assert_allclose(paddle.linalg.slogdet(P(m)).numpy().reshape(-1), [sgn, logdet], rtol=1e-8)
    np.testing.assert_allclose(paddle.linalg.matrix_power(P(m), 3).numpy(), np.linalg.matrix_power(m, 3), rtol=1e-8)
    np.testing.assert_allclose(paddle.linalg.pinv(P(U(5, 3))).numpy() @ np.eye(5)[:, :5].T.T[:5, :5] is not None, True)
    x = U(5, 3)
    np.testing.assert_allclose(paddle.linalg.pinv(P(x)).numpy(), np.linalg.pinv(x), rtol=1e-6, atol=1e-8)
    np.testing.assert_allclose(paddle.t(P(x)).numpy(), x.T)
    np.testing.assert_allclose(paddle.trace(P(m)).numpy().reshape(-1), [np.trace(m)])
    np.testing.assert_allclose(paddle.kron(P(c1[:2, :2]), P(c2[:2, :2])).numpy(), np.kron(c1[:2, :2], c2[:2, :2]))


# ----------------------------------------------------------------------------- losses
def test_losses():
    F = paddle.nn.functional
    x, y = U(6, 5), U(6, 5)
    np.testing.assert_allclose(F.mse_loss(P(x), P(y)).numpy().reshape(-1), [np.mean((x - y) ** 2)])
    np.testing.assert_allclose(F.l1_loss(P(x), P(y), reduction="sum").numpy().reshape(-1), [np.abs(x - y).sum()])
    # smooth_l1 is the Huber form with delta (test_smooth_l1_loss.py smooth_l1_loss_forward)
    for delta in (1.0, 0.3):
        d = x - y
        ref = np.where(np.abs(d) <= delta, 0.5 * d * d, delta * (np.abs(d) - 0.5 * delta)).mean()
        np.testing.assert_allclose(F.smooth_l1_loss(P(x), P(y), delta=delta).numpy().reshape(-1), [ref], rtol=1e-7)
    logits = U(6, 5, lo=-3, hi=3)
    lab = R.randint(0, 5, (6,))
    lp = np.log(softmax_np(logits))
    np.testing.assert_allclose(F.cross_entropy(P(logits), P(lab)).numpy().reshape(-1),
                               [-lp[np.arange(6), lab].mean()], rtol=1e-7)
    # ignore_index + class weights: mean over the weights of non-ignored samples (test_cross_entropy_loss.py)
    lab2 = lab.copy()
    lab2[1] = -100
    w = R.uniform(0.5, 2, 5)
    keep = lab2 != -100
    num = -(w[lab2[keep]] * lp[np.arange(6)[keep], lab2[keep]]).sum()
    np.testing.assert_allclose(F.cross_entropy(P(logits), P(lab2), weight=P(w), ignore_index=-100).numpy().reshape(-1),
                               [num / w[lab2[keep]].sum()], rtol=1e-7)
    soft = softmax_np(U(6, 5))
    np.testing.assert_allclose(F.cross_entropy(P(logits), P(soft), soft_label=True).numpy().reshape(-1),
                               [-(soft * lp).sum(1).mean()], rtol=1e-7)
    np.testing.assert_allclose(F.nll_loss(P(lp), P(lab)).numpy().reshape(-1), [-lp[np.arange(6), lab].mean()])
    p = U(6, 5, lo=0.05, hi=0.95)
    t = (U(6, 5) > 0).astype("float64")
    np.testing.assert_allclose(F.binary_cross_entropy(P(p), P(t)).numpy().reshape(-1),
                               [-(t * np.log(p) + (1 - t) * np.log(1 - p)).mean()], rtol=1e-7)
    pw = R.uniform(0.5, 2, 5)
    sig = 1 / (1 + np.exp(-logits))
    ref = -(pw * t * np.log(sig) + (1 - t) * np.log(1 - sig)).mean()
    np.testing.assert_allclose(F.binary_cross_entropy_with_logits(P(logits), P(t), pos_weight=P(pw)).numpy().reshape(-1),
                               [ref], rtol=1e-7)
    q = softmax_np(U(6, 5))
    # kl_div(input=log-probs, label=probs), reduction 'mean' averages over all elements (test_kldiv_loss_op.py)
    np.testing.assert_allclose(F.kl_div(P(lp), P(q)).numpy().reshape(-1), [(q * (np.log(q) - lp)).mean()], rtol=1e-7)
    a, b, l = U(6), U(6), np.sign(U(6))
    np.testing.assert_allclose(F.margin_ranking_loss(P(a), P(b), P(l), margin=0.1).numpy().reshape(-1),
                               [np.maximum(0, -l * (a - b) + 0.1).mean()], rtol=1e-7)
    e1, e2 = U(4, 6), U(4, 6)
    cos = (e1 * e2).sum(1) / np.linalg.norm(e1, axis=1) / np.linalg.norm(e2, axis=1)
    np.testing.assert_allclose(F.cosine_similarity(P(e1), P(e2), axis=1).numpy(), cos, rtol=1e-7)
    ls = F.label_smooth(P(np.eye(5)[lab]), epsilon=0.1).numpy()
    np.testing.assert_allclose(ls, 0.9 * np.eye(5)[lab] + 0.1 / 5)
    hl = F.hinge_embedding_loss(P(a), P(l), margin=1.0).numpy().reshape(-1) if hasattr(F, "hinge_embedding_loss") else None
    if hl is not None:
        np.testing.assert_allclose(hl, [np.where(l == 1, a, np.maximum(0, 1.0 - a)).mean()], rtol=1e-7)


# ----------------------------------------------------------------------------- nn functional
def test_norms():
    F = paddle.nn.functional
    x = U(2, 3, 4, 5)
    w, b = U(5) + 1, U(5)
    mu = x.mean(-1, keepdims=True)
    var = x.var(-1, keepdims=True)
    np.testing.assert_allclose(F.layer_norm(P(x), 5, P(w), P(b), 1e-5).numpy(), (x - mu) / np.sqrt(var + 1e-5) * w + b,
                               rtol=1e-6)
    rm, rv, g, bb = U(3), U(3, lo=0.5, hi=2), U(3), U(3)
    ref = (x - rm[:, None, None]) / np.sqrt(rv[:, None, None] + 1e-5) * g[:, None, None] + bb[:, None, None]
    np.testing.assert_allclose(F.batch_norm(P(x), P(rm), P(rv), P(g), P(bb), training=False).numpy(), ref, rtol=1e-6)
    mu = x.mean((2, 3), keepdims=True)
    var = x.var((2, 3), keepdims=True)
    np.testing.assert_allclose(F.instance_norm(P(x)).numpy(), (x - mu) / np.sqrt(var + 1e-5), rtol=1e-5, atol=1e-6)
    xg = x.reshape(2, 3, -1)
    gn = (xg - xg.mean(-1, keepdims=True)) / np.sqrt(xg.var(-1, keepdims=True) + 1e-5)
    np.testing.assert_allclose(F.group_norm(P(x), 3).numpy() if hasattr(F, "group_norm") else
                               paddle.nn.GroupNorm(3, 3)(P(x)).numpy(), gn.reshape(x.shape), rtol=1e-5, atol=1e-6)
    nrm = F.normalize(P(x), p=2, axis=1).numpy()
    np.testing.assert_allclose(nrm, x / np.maximum(np.linalg.norm(x, axis=1, keepdims=True), 1e-12), rtol=1e-7)


def test_conv_pool_pad():
    F = paddle.nn.functional
    x = U(2, 3, 7, 7)
    w = U(4, 3, 3, 3)

    def conv_np(x, w, stride=1, pad=0, dil=1):
        xp = np.pad(x, ((0, 0), (0, 0), (pad, pad), (pad, pad)))
        kh = (w.shape[2] - 1) * dil + 1
        oh = (xp.shape[2] - kh) // stride + 1
        out = np.zeros((x.shape[0], w.shape[0], oh, oh))
        for i in range(oh):
            for j in range(oh):
                patch = xp[:, :, i * stride:i * stride + kh:dil, j * stride:j * stride + kh:dil]
                out[:, :, i, j] = np.tensordot(patch, w, ([1, 2, 3], [1, 2, 3]))
        return out
    np.testing.assert_allclose(F.conv2d(P(x), P(w), stride=2, padding=1).numpy(), conv_np(x, w, 2, 1), rtol=1e-7)
    np.testing.assert_allclose(F.conv2d(P(x), P(w), dilation=2).numpy(), conv_np(x, w, 1, 0, 2), rtol=1e-7)
    mp = F.max_pool2d(P(x), 2, 2).numpy()
    np.testing.assert_allclose(mp, x[:, :, :6, :6].reshape(2, 3, 3, 2, 3, 2).max((3, 5)))
    # avg pool with padding: exclusive=True (default) divides by the in-bounds count (test_pool2d_op.py)
    ap = F.avg_pool2d(P(x), 3, 2, padding=1).numpy()
    xp = np.pad(x, ((0, 0), (0, 0), (1, 1), (1, 1)))
    ones = np.pad(np.ones_like(x), ((0, 0), (0, 0), (1, 1), (1, 1)))
    ref = np.zeros_like(ap)
    for i in range(ap.shape[2]):
        for j in range(ap.shape[3]):
            s = xp[:, :, 2 * i:2 * i + 3, 2 * j:2 * j + 3].sum((2, 3))
            n = ones[:, :, 2 * i:2 * i + 3, 2 * j:2 * j + 3].sum((2, 3))
            ref[:, :, i, j] = s / n
    np.testing.assert_allclose(ap, ref, rtol=1e-7)
    ap_inc = F.avg_pool2d(P(x), 3, 2, padding=1, exclusive=False).numpy()
    np.testing.assert_allclose(ap_inc[:, :, 0, 0], xp[:, :, :3, :3].sum((2, 3)) / 9, rtol=1e-7)
    np.testing.assert_allclose(F.adaptive_avg_pool2d(P(x), 1).numpy(), x.mean((2, 3), keepdims=True), rtol=1e-7)
    np.testing.assert_allclose(F.pad(P(x), [1, 2, 0, 1], mode="constant", value=0.5).numpy(),
                               np.pad(x, ((0, 0), (0, 0), (0, 1), (1, 2)), constant_values=0.5))
    np.testing.assert_allclose(F.pad(P(x), [1, 1, 2, 2], mode="reflect").numpy(),
                               np.pad(x, ((0, 0), (0, 0), (2, 2), (1, 1)), mode="reflect"))
    np.testing.assert_allclose(F.pad(P(x), [1, 1, 2, 2], mode="replicate").numpy(),
                               np.pad(x, ((0, 0), (0, 0), (2, 2), (1, 1)), mode="edge"))
    np.testing.assert_allclose(F.pad(P(x), [1, 1, 2, 2], mode="circular").numpy(),
                               np.pad(x, ((0, 0), (0, 0), (2, 2), (1, 1)), mode="wrap"))
    ps = F.pixel_shuffle(P(U(1, 8, 2, 3)), 2).numpy()
    assert ps.shape == (1, 2, 4, 6)
    up = F.interpolate(P(x), scale_factor=2, mode="nearest").numpy()
    np.testing.assert_allclose(up, x.repeat(2, 2).repeat(2, 3))
    e = U(10, 4)
    ids = np.array([[1, 0], [9, 1]])
    np.testing.assert_allclose(F.embedding(P(ids), P(e)).numpy(), e[ids])
    out = F.embedding(P(ids), P(e), padding_idx=0).numpy()
    np.testing.assert_allclose(out[0, 1], np.zeros(4))
    np.testing.assert_allclose(F.dropout(P(x), 0.3, training=False).numpy(), x)   # upscale_in_train: identity at eval
    np.testing.assert_allclose(F.dropout(P(x), 0.3, training=False, mode="downscale_in_infer").numpy(), x * 0.7)
    np.testing.assert_allclose(paddle.clip(P(x), -0.2, 0.3).numpy(), np.clip(x, -0.2, 0.3))
    np.testing.assert_allclose(F.linear(P(U(3, 4)), P(w.reshape(4, -1)[:, :5] if False else U(4, 5))).numpy().shape, (3, 5))


# ----------------------------------------------------------------------------- batch 2 (less common ops)
def test_renorm_fixture():
    # test_renorm_op.py: values and expected output copied from the reference test's fixture
    x = np.array([[[2.0, 2, -2], [3, 0.3, 3]], [[2, -8, 2], [3.1, 3.7, 3]]])
    expected = np.array([[[0.40594056, 0.29285714, -0.41000000], [0.60891086, 0.04392857, 0.61500001]],
                         [[0.40594056, -1.17142856, 0.41000000], [0.62920785, 0.54178572, 0.61500001]]])
    np.testing.assert_allclose(paddle.renorm(P(x), 1.0, 2, 2.05).numpy(), expected, rtol=1e-6)


def test_sigmoid_focal_loss():
    # test_sigmoid_focal_loss.py calc_sigmoid_focal_loss
    F = paddle.nn.functional
    logit = U(5, 3, lo=-3, hi=3)
    label = (U(5, 3) > 0).astype("float64")
    norm = np.array([2.5])
    loss = np.maximum(logit, 0) - logit * label + np.log(1 + np.exp(-np.abs(logit)))
    pred = 1 / (1 + np.exp(-logit))
    p_t = pred * label + (1 - pred) * (1 - label)
    loss = (0.25 * label + 0.75 * (1 - label)) * loss * (1 - p_t) ** 2.0 / norm
    np.testing.assert_allclose(F.sigmoid_focal_loss(P(logit), P(label), P(norm), reduction="sum").numpy().reshape(-1),
                               [loss.sum()], rtol=1e-6)
    np.testing.assert_allclose(F.sigmoid_focal_loss(P(logit), P(label), P(norm), reduction="none").numpy(), loss,
                               rtol=1e-6)


def test_log_loss_and_square_error():
    F = paddle.nn.functional
    pred = 1 / (1 + np.exp(-U(10, 1)))
    lab = (U(10, 1) > 0).astype("float64")
    want = -lab * np.log(pred + 1e-4) - (1 - lab) * np.log(1 - pred + 1e-4)     # test_log_loss_op.py
    np.testing.assert_allclose(F.log_loss(P(pred), P(lab), epsilon=1e-4).numpy(), want, rtol=1e-6)
    a, b = U(4, 3), U(4, 3)
    np.testing.assert_allclose(F.square_error_cost(P(a), P(b)).numpy(), (a - b) ** 2)


def test_temporal_shift():
    # test_temporal_shift_op.py temporal_shift
    x = U(6, 4, 2, 2)
    seg, ratio = 3, 0.25
    shape = x.shape
    r = x.reshape((-1, seg) + shape[1:])
    pad = np.pad(r, ((0, 0), (1, 1), (0, 0), (0, 0), (0, 0)))
    c1, c2 = int(shape[1] * ratio), int(shape[1] * 2 * ratio)
    want = np.concatenate([pad[:, :seg, :c1], pad[:, 2:seg + 2, c1:c2], pad[:, 1:seg + 1, c2:]], 2).reshape(shape)
    np.testing.assert_allclose(paddle.nn.functional.temporal_shift(P(x), seg, ratio).numpy(), want)


def test_gather_tree_backtrace():
    # test_gather_tree_op.py backtrace
    ids = R.randint(0, 10, (5, 2, 3)).astype("int64")
    parents = R.randint(0, 3, (5, 2, 3)).astype("int64")
    T, B, K = ids.shape
    want = np.zeros_like(ids)
    for b in range(B):
        for k in range(K):
            want[T - 1, b, k] = ids[T - 1, b, k]
            p = parents[T - 1, b, k]
            for t in range(T - 2, -1, -1):
                want[t, b, k] = ids[t, b, p]
                p = parents[t, b, p]
    np.testing.assert_array_equal(paddle.nn.functional.gather_tree(P(ids), P(parents)).numpy(), want)


def test_multiplex_and_misc_math():
    rows = 4
    index = np.array([[2], [0], [3], [1]], dtype="int32")
    ins = [U(rows, 5) for _ in range(4)]
    want = np.stack([ins[index[i, 0]][i] for i in range(rows)])            # test_multiplex_op.py
    np.testing.assert_allclose(paddle.multiplex([P(t) for t in ins], P(index)).numpy(), want)
    a, b = U(3, 4), U(3, 4)
    np.testing.assert_allclose(paddle.lerp(P(a), P(b), 0.3).numpy(), a + 0.3 * (b - a))
    np.testing.assert_allclose(paddle.diff(P(a), axis=1).numpy(), np.diff(a, axis=1))
    np.testing.assert_allclose(paddle.rot90(P(a), 1, [0, 1]).numpy(), np.rot90(a, 1, (0, 1)))
    np.testing.assert_allclose(paddle.inner(P(a), P(b)).numpy(), np.inner(a, b))
    np.testing.assert_allclose(paddle.outer(P(a[0]), P(b[0])).numpy(), np.outer(a[0], b[0]))
    np.testing.assert_allclose(paddle.addmm(P(a[:, :3]), P(a), P(b.T[:, :3])).numpy(), a[:, :3] + a @ b.T[:, :3])
    gi, gj = np.array([12, 18, -9]), np.array([8, 12, 6])
    np.testing.assert_array_equal(paddle.gcd(P(gi), P(gj)).numpy(), np.gcd(gi, gj))
    np.testing.assert_array_equal(paddle.lcm(P(gi), P(gj)).numpy(), np.lcm(gi, gj))
    np.testing.assert_allclose(paddle.quantile(P(a), 0.3, axis=1).numpy(), np.quantile(a, 0.3, axis=1))
    np.testing.assert_allclose(paddle.frac(P(a * 5)).numpy(), np.modf(a * 5)[0])
    np.testing.assert_allclose(paddle.diagflat(P(a[0])).numpy(), np.diagflat(a[0]))
    np.testing.assert_allclose(paddle.erfinv(P(x_unit)).numpy(),
                               np.vectorize(lambda v: _erfinv(v))(x_unit), rtol=1e-6, atol=1e-8)
    np.testing.assert_allclose(paddle.angle(P(np.array([1 + 1j, -1 + 0j, 0 - 2j]))).numpy(),
                               np.angle(np.array([1 + 1j, -1 + 0j, 0 - 2j])))


def _erfinv(y):
    # Newton on erf (no scipy): erf'(x) = 2/sqrt(pi) exp(-x^2)
    x = 0.0
    for _ in range(60):
        x -= (math.erf(x) - y) / (2 / math.sqrt(math.pi) * math.exp(-x * x))
    return x


def test_sequence_mask_channel_shuffle_unfold():
    F = paddle.nn.functional
    lens = np.array([1, 3, 0, 2])
    want = (np.arange(4)[None, :] < lens[:, None]).astype("int64")
    np.testing.assert_array_equal(F.sequence_mask(P(lens), maxlen=4).numpy(), want)
    x = U(2, 6, 3, 3)
    g = 3
    want = x.reshape(2, g, 2, 3, 3).transpose(0, 2, 1, 3, 4).reshape(2, 6, 3, 3)   # test_channel_shuffle.py
    np.testing.assert_allclose(F.channel_shuffle(P(x), g).numpy(), want)
    # unfold (im2col): [N, C*kh*kw, L] (test_unfold_op.py)
    xx = U(1, 2, 4, 4)
    cols = F.unfold(P(xx), [2, 2], strides=2).numpy()
    want = np.stack([xx[0, :, i:i + 2, j:j + 2].reshape(-1) for i in (0, 2) for j in (0, 2)], 1)[None]
    np.testing.assert_allclose(cols, want)
    np.testing.assert_allclose(F.pixel_shuffle(F.pixel_unshuffle(P(x[:, :4]), 1), 1).numpy(), x[:, :4]) \
        if hasattr(F, "pixel_unshuffle") else None


def test_margin_and_hinge_losses():
    F = paddle.nn.functional
    a = U(6, 4)
    lab = np.sign(U(6, 4))
    # soft_margin_loss: mean(log(1 + exp(-y x))) (reference nn/functional/loss.py soft_margin_loss)
    if hasattr(F, "soft_margin_loss"):
        np.testing.assert_allclose(F.soft_margin_loss(P(a), P(lab)).numpy().reshape(-1),
                                   [np.log(1 + np.exp(-lab * a)).mean()], rtol=1e-6)
    # npair_loss (test_npair_loss_op.py): softmax CE over anchor.positive^T + l2 reg
    anchor, pos = U(4, 3), U(4, 3)
    labels = np.array([0, 1, 2, 1]).astype("float64")
    l2 = 0.002
    sim = anchor @ pos.T
    same = (labels[:, None] == labels[None, :]).astype("float64")
    tgt = same / same.sum(1, keepdims=True)
    ce = -(tgt * np.log(softmax_np(sim))).sum(1).mean()
    reg = l2 * 0.25 * ((anchor ** 2).sum(1).mean() + (pos ** 2).sum(1).mean())
    np.testing.assert_allclose(F.npair_loss(P(anchor), P(pos), P(labels), l2_reg=l2).numpy().reshape(-1),
                               [ce + reg], rtol=1e-6)


# ----------------------------------------------------------------------------- batch 3 (search / stat / shape ops)
def test_logcumsumexp_and_cummax():
    # test_logcumsumexp_op.py np_logcumsumexp; test_cummax_op.py cummax_dim
    x = U(3, 5)
    want = np.log(np.cumsum(np.exp(x), axis=1))
    np.testing.assert_allclose(paddle.logcumsumexp(P(x), axis=1).numpy(), want, rtol=1e-6)
    if hasattr(paddle, "cummax"):
        v, i = paddle.cummax(P(x), axis=1)
        np.testing.assert_allclose(v.numpy(), np.maximum.accumulate(x, axis=1))


def test_bincount_histogram_searchsorted_bucketize():
    ints = R.randint(0, 6, (20,)).astype("int64")
    w = U(20)
    np.testing.assert_array_equal(paddle.bincount(P(ints)).numpy(), np.bincount(ints))       # test_bincount_op.py
    np.testing.assert_allclose(paddle.bincount(P(ints), weights=P(w)).numpy(), np.bincount(ints, weights=w))
    xs = U(50, lo=0, hi=10)
    # test_histogram_op.py: np.histogram(x, bins, range=(min, max)), int64 counts
    np.testing.assert_array_equal(paddle.histogram(P(xs), bins=5, min=0, max=10).numpy(),
                                  np.histogram(xs, 5, range=(0, 10))[0])
    seq = np.sort(U(10))
    vals = U(6)
    for right in (False, True):   # test_searchsorted_op.py
        np.testing.assert_array_equal(paddle.searchsorted(P(seq), P(vals), right=right).numpy(),
                                      np.searchsorted(seq, vals, side="right" if right else "left"))
        np.testing.assert_array_equal(paddle.bucketize(P(vals), P(seq), right=right).numpy(),
                                      np.searchsorted(seq, vals, side="right" if right else "left"))


def test_trace_kron_cross_dist():
    a = U(4, 5)
    for off in (-1, 0, 2):   # test_trace_op.py
        np.testing.assert_allclose(paddle.trace(P(a), offset=off).numpy().reshape(-1), [np.trace(a, offset=off)])
    b = U(2, 3)
    np.testing.assert_allclose(paddle.kron(P(a), P(b)).numpy(), np.kron(a, b))              # test_kron_op.py
    u, v = U(4, 3), U(4, 3)
    np.testing.assert_allclose(paddle.cross(P(u), P(v), axis=1).numpy(), np.cross(u, v, axis=1))
    for p in (1.0, 2.0, float("inf"), 0.0):   # test_dist_op.py: norm of the difference
        want = (np.count_nonzero(u - v) if p == 0 else np.max(np.abs(u - v)) if p == float("inf")
                else (np.abs(u - v) ** p).sum() ** (1 / p))
        np.testing.assert_allclose(paddle.dist(P(u), P(v), p).numpy().reshape(-1), [want], rtol=1e-6)


def test_take_put_along_axis_index_sample_masked_select():
    x = U(3, 4)
    idx = R.randint(0, 4, (3, 2)).astype("int64")
    np.testing.assert_allclose(paddle.take_along_axis(P(x), P(idx), 1).numpy(), np.take_along_axis(x, idx, 1))
    vals = U(3, 2)
    want = x.copy()
    np.put_along_axis(want, idx, vals, 1)                                      # test_put_along_axis_op.py
    got = paddle.put_along_axis(P(x), P(idx), P(vals), 1).numpy()
    # duplicate indices in a row: the reference kernel's last write wins, like numpy's
    np.testing.assert_allclose(got, want)
    # index_sample (test_index_sample_op.py): out[i][j] = x[i][index[i][j]]
    np.testing.assert_allclose(paddle.index_sample(P(x), P(idx)).numpy(), np.take_along_axis(x, idx, 1))
    m = x > 0
    np.testing.assert_allclose(paddle.masked_select(P(x), P(m)).numpy(), x[m])


def test_unique_family_roll_flip_tri():
    a = R.randint(0, 5, (12,)).astype("int64")
    out, idx, inv, cnt = paddle.unique(P(a), return_index=True, return_inverse=True, return_counts=True)
    wo, wi, winv, wc = np.unique(a, return_index=True, return_inverse=True, return_counts=True)   # test_unique.py
    for g, w in ((out, wo), (idx, wi), (inv, winv), (cnt, wc)):
        np.testing.assert_array_equal(g.numpy(), w)
    b = np.array([1, 1, 2, 2, 2, 3, 1, 1], dtype="int64")
    uc, ucnt = paddle.unique_consecutive(P(b), return_counts=True)
    np.testing.assert_array_equal(uc.numpy(), [1, 2, 3, 1])                     # test_unique_consecutive_op.py
    np.testing.assert_array_equal(ucnt.numpy(), [2, 3, 1, 2])
    x = U(3, 4)
    np.testing.assert_allclose(paddle.roll(P(x), 1, axis=1).numpy(), np.roll(x, 1, axis=1))
    np.testing.assert_allclose(paddle.roll(P(x), 5).numpy(), np.roll(x, 5))    # flattened roll
    np.testing.assert_allclose(paddle.flip(P(x), [0, 1]).numpy(), np.flip(x, (0, 1)))
    for d in (-1, 0, 1):
        np.testing.assert_allclose(paddle.tril(P(x), d).numpy(), np.tril(x, d))
        np.testing.assert_allclose(paddle.triu(P(x), d).numpy(), np.triu(x, d))


def test_creation_ranges():
    np.testing.assert_allclose(paddle.linspace(0, 1, 7).numpy(), np.linspace(0, 1, 7).astype("float32"), rtol=1e-6)
    np.testing.assert_allclose(paddle.logspace(0, 2, 5, base=10.0).numpy(),
                               np.logspace(0, 2, 5).astype("float32"), rtol=1e-5)
    np.testing.assert_array_equal(paddle.arange(2, 11, 3).numpy(), np.arange(2, 11, 3))
    e = paddle.eye(3, 4).numpy()
    np.testing.assert_array_equal(e, np.eye(3, 4))
    g1, g2 = paddle.meshgrid(P(np.arange(3.0)), P(np.arange(4.0)))
    w1, w2 = np.meshgrid(np.arange(3.0), np.arange(4.0), indexing="ij")          # paddle meshgrid is 'ij'
    np.testing.assert_array_equal(g1.numpy(), w1)
    np.testing.assert_array_equal(g2.numpy(), w2)
    v = U(3)
    np.testing.assert_allclose(paddle.diag_embed(P(v)).numpy(), np.diag(v))
    np.testing.assert_array_equal(paddle.nonzero(P(np.array([[0, 1], [2, 0]]))).numpy(), [[0, 1], [1, 0]])


def test_stat_cov_corrcoef_mode_nanmedian():
    x = U(3, 6)
    if hasattr(paddle.linalg, "cov"):
        np.testing.assert_allclose(paddle.linalg.cov(P(x)).numpy(), np.cov(x), rtol=1e-6)
    if hasattr(paddle.linalg, "corrcoef"):
        np.testing.assert_allclose(paddle.linalg.corrcoef(P(x)).numpy(), np.corrcoef(x), rtol=1e-6)
    y = x.copy()
    y[0, 1] = np.nan
    if hasattr(paddle, "nanmedian"):
        # test_nanmedian.py: np.nanmedian (even counts average the two middle values)
        np.testing.assert_allclose(paddle.nanmedian(P(y), axis=1, keepdim=False).numpy(), np.nanmedian(y, axis=1))
        np.testing.assert_allclose(paddle.nanmedian(P(y), axis=[0, 1]).numpy().reshape(-1), [np.nanmedian(y)])
        np.testing.assert_allclose(paddle.nanmedian(P(y)).numpy().reshape(-1), [np.nanmedian(y)])
    np.testing.assert_allclose(paddle.nansum(P(y), axis=1).numpy(), np.nansum(y, axis=1))


def test_clip_increment_scale_stanh():
    x = U(4, 5, lo=-3, hi=3)
    np.testing.assert_allclose(paddle.clip(P(x), -1.5, 0.7).numpy(), np.clip(x, -1.5, 0.7))
    np.testing.assert_allclose(paddle.increment(P(np.array([3.0])), 2.5).numpy(), [5.5])
    # scale_op: bias_after_scale True: x * s + b, False: (x + b) * s (test_scale_op.py)
    np.testing.assert_allclose(paddle.scale(P(x), 2.0, 0.5, bias_after_scale=True).numpy(), x * 2 + 0.5)
    np.testing.assert_allclose(paddle.scale(P(x), 2.0, 0.5, bias_after_scale=False).numpy(), (x + 0.5) * 2)


def test_pairwise_distance():
    # test_pairwise_distance.py: np.linalg.norm(x - y, ord=p, axis=1, keepdims=keepdim)
    x, y = U(5, 4), U(5, 4)
    for p in (1.0, 2.0, 3.0, float("inf"), 0.0):
        for keep in (False, True):
            got = paddle.nn.functional.pairwise_distance(P(x), P(y), p=p, keepdim=keep).numpy()
            np.testing.assert_allclose(got, np.linalg.norm(x - y, ord=p, axis=1, keepdims=keep), rtol=1e-6)
            np.testing.assert_allclose(paddle.nn.PairwiseDistance(p=p, keepdim=keep)(P(x), P(y)).numpy(), got)


def _log_softmax_np(x, axis=-1):
    return np.log(softmax_np(x, axis))


@pytest.mark.parametrize("reduction", ["mean", "sum", "none"])
def test_cross_entropy_hard_weighted_ignore(reduction):
    # test_cross_entropy_loss.py cross_entropy_loss_1d
    x = U(8, 5)
    lab = R.randint(0, 5, (8,)).astype("int64")
    lab[2] = -100
    w = U(5, lo=0.2, hi=2.0)
    ls = _log_softmax_np(x)
    out = np.array([0.0 if lab[i] == -100 else -ls[i, lab[i]] * w[lab[i]] for i in range(8)])
    tw = sum(w[lab[i]] for i in range(8) if lab[i] != -100)
    want = out.sum() / tw if reduction == "mean" else out.sum() if reduction == "sum" else out
    got = paddle.nn.functional.cross_entropy(P(x), P(lab), weight=P(w), reduction=reduction).numpy()
    np.testing.assert_allclose(got.reshape(np.shape(want)), want, rtol=1e-6)


@pytest.mark.parametrize("reduction", ["mean", "sum", "none"])
def test_cross_entropy_soft_weighted(reduction):
    # test_cross_entropy_loss.py cross_entropy_soft: per-sample weight = dot(weight, soft label)
    x = U(6, 4)
    lab = softmax_np(U(6, 4) * 3)
    w = U(4, lo=0.2, hi=2.0)
    loss = (-lab * _log_softmax_np(x)).sum(-1, keepdims=True)
    cw = lab @ w
    wl = loss * cw[:, None]
    want = wl.sum() / cw.sum() if reduction == "mean" else wl.sum() if reduction == "sum" else wl
    got = paddle.nn.functional.cross_entropy(P(x), P(lab), soft_label=True, weight=P(w), reduction=reduction).numpy()
    np.testing.assert_allclose(got.reshape(np.shape(want)), want, rtol=1e-6)


def test_cross_entropy_soft_unweighted_none_keeps_dim():
    x = U(6, 4)
    lab = softmax_np(U(6, 4))
    want = (-lab * _log_softmax_np(x)).sum(-1, keepdims=True)
    got = paddle.nn.functional.cross_entropy(P(x), P(lab), soft_label=True, reduction="none").numpy()
    np.testing.assert_allclose(got.reshape(want.shape), want, rtol=1e-6)


@pytest.mark.parametrize("reduction", ["batchmean", "mean", "sum", "none"])
def test_kl_div_negative_targets_masked(reduction):
    # test_kldiv_loss_op.py kldiv_loss: elements with target < 0 contribute 0
    x = U(5, 6, lo=-10, hi=10)
    t = U(5, 6, lo=-10, hi=10)
    with np.errstate(invalid="ignore"):
        out = np.where(t >= 0, t * (np.log(t) - x), 0.0)
    want = {"batchmean": out.sum() / 5, "mean": out.mean(), "sum": out.sum(), "none": out}[reduction]
    got = paddle.nn.functional.kl_div(P(x), P(t), reduction=reduction).numpy()
    np.testing.assert_allclose(got.reshape(np.shape(want)), want, rtol=1e-6)


def test_conv3d_depth_tap_decomposition(monkeypatch):
    """the GPU route of conv3d (one 2-D convolution per depth tap, nn/functional/conv.py
    _conv3d_as_2d) checked on CPU with a plain NHWC 2-D convolution standing in for the own kernel"""
    import torch
    import torch.nn.functional as TF
    from paddle_hackathon_amd.nn.functional import conv as C

    def fake_own(t, w, bias, stride, padding, dilation, groups, data_format):
        y = TF.conv2d(t.permute(0, 3, 1, 2), w, None, stride, padding, dilation, groups)
        return y.permute(0, 2, 3, 1)
    monkeypatch.setattr(C, "_own_conv2d", fake_own)
    torch.manual_seed(0)
    x = torch.randn(2, 4, 7, 6, 5, dtype=torch.float64)
    w = torch.randn(6, 4, 3, 2, 3, dtype=torch.float64)
    b = torch.randn(6, dtype=torch.float64)
    for fmt in ("NCDHW", "NDHWC"):
        xin = x.permute(0, 2, 3, 4, 1) if fmt == "NDHWC" else x
        out = C._conv3d_as_2d(xin, w, b, [2, 1, 2], [1, 0, 1], [1, 1, 1], 1, fmt)
        ref = TF.conv3d(x, w, b, [2, 1, 2], [1, 0, 1])
        if fmt == "NDHWC":
            out = out.permute(0, 4, 1, 2, 3)
        torch.testing.assert_close(out, ref)
    out = C._conv3d_as_2d(x, w, None, 1, 2, [2, 1, 1], 1, "NCDHW")
    torch.testing.assert_close(out, TF.conv3d(x, w, None, 1, 2, [2, 1, 1]))


def test_grouped_conv_merge_is_block_diagonal():
    """ops/conv_gemm.py _merge_groups: m narrow groups merged into one with block-diagonal filters
    compute the same convolution (what lets cig = 4 groups run on the grouped MFMA GEMM)"""
    import torch
    import torch.nn.functional as TF
    from paddle_hackathon_amd.ops.conv_gemm import _merge_groups, _merge_factor
    torch.manual_seed(0)
    x = torch.randn(2, 128, 7, 7, dtype=torch.float64)
    w = torch.randn(128, 4, 3, 3, dtype=torch.float64)
    m = _merge_factor(4, 4, 32)
    assert m == 2
    ref = TF.conv2d(x, w, padding=1, groups=32)
    got = TF.conv2d(x, _merge_groups(w, 32, m), padding=1, groups=16)
    torch.testing.assert_close(got, ref)
    assert _merge_factor(8, 8, 32) == 1 and _merge_factor(2, 2, 32) == 4 and _merge_factor(3, 3, 5) is None
