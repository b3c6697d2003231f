"""Host side of the gfx950 MFMA GEMM / implicit-GEMM convolution (csrc/kernels/gemm_conv.hip).

``conv2d_nhwc`` is an autograd Function whose forward, data-gradient and weight-gradient
are all the same MFMA kernel with different operand loaders:

  * forward   : out[(n,oh,ow), co] = im2col(x)[m, (kh,kw,ci)] @ W^T          (A_CONV x B_ROW)
  * grad data : stride 1 — the forward kernel on dY with the spatially flipped, channel-
                transposed kernel; stride s — s*s sub-pixel convolutions (one per output
                phase, each a stride-1 conv over dY with that phase's taps), interleaved.
  * grad wgt  : dW[co, (kh,kw,ci)] = dY^T @ im2col(x), reduction over N*OH*OW output pixels,
                split-K across blocks with an fp32 slab reduction             (A_COL x B_CONV)

Layouts: activations NHWC (C contiguous), weights Paddle OIHW [Cout, Cin, KH, KW].
Requires bf16/fp16, Cin % 8 == 0 and Cout % 8 == 0 (everything in ResNet after the stem);
other shapes use the portable path in nn.functional.conv.
"""
from __future__ import annotations

import ctypes
from ctypes import byref, c_int, c_long, c_void_p

import json
import os

import torch

from . import _lib

A_ROW, A_COL, A_CONV = 0, 1, 2
B_ROW, B_COL, B_CONV = 0, 1, 2
EPI = {None: 0, "relu": 1, "gelu": 2}
_DT = {torch.bfloat16: 1, torch.float16: 2}
_sig = False
_zero = {}


def _L():
    global _sig
    L = _lib.lib
    if L is None:
        raise RuntimeError("libpha_kernels.so not loaded")
    if not _sig:
        P, I, LG = c_void_p, c_int, c_long
        L.pha_gemm.argtypes = [I, I, I, I, P, LG, P, LG, P, LG, P, LG, LG, LG, I, P, P, P, P]
        L.pha_gemm.restype = c_int
        _sig = True
    return L


def _ptr(t):
    return c_void_p(0 if t is None else t.data_ptr())


def _zero_page(dev):
    z = _zero.get(dev)
    if z is None:
        z = torch.zeros(256, dtype=torch.uint8, device=dev)
        _zero[dev] = z
    return z


def _num_cus(dev):
    return torch.cuda.get_device_properties(dev).multi_processor_count


def _pick_splitk(M, N, K, dev, force=None):
    if force is not None:
        return max(1, int(force))
    # enough (tile x K-slice) blocks to cover every CU twice; each slice keeps >= 256 of K
    tiles = ((M + 127) // 128) * ((N + 127) // 128)
    target = 2 * _num_cus(dev)
    if tiles >= target or K < 1024:
        return 1
    s = min((target + tiles - 1) // tiles, K // 256, 1024)
    return max(1, s)


def gemm_raw(amode, bmode, a, lda, b, ldb, c, ldc, M, N, K, bias=None, act=None, conv=None, splitk=None):
    """Launch one GEMM; all tensors must already have the layouts the modes describe."""
    dev = c.device
    sk = _pick_splitk(M, N, K, dev, splitk)
    ws = torch.empty(sk * M * N, dtype=torch.float32, device=dev) if sk > 1 else None
    cv = None
    if conv is not None:
        cv = (ctypes.c_int * 14)(*conv)
    stream = c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    rc = _L().pha_gemm(_DT[c.dtype], amode, bmode, EPI[act], _ptr(a), lda, _ptr(b), ldb, _ptr(c), ldc,
                       _ptr(bias), M, N, K, sk, _ptr(ws), cv, _ptr(_zero_page(dev)), stream)
    if rc != 0:
        raise RuntimeError(f"pha_gemm failed (hip error {rc}) M={M} N={N} K={K} modes=({amode},{bmode})")
    return c


# ----------------------------------------------------------------------------- dense matmul
def matmul(a, b, trans_a=False, trans_b=False, bias=None, act=None):
    """2-D bf16/fp16 matmul on the MFMA kernel: op(a) @ op(b) (+bias) (+act)."""
    assert a.dim() == 2 and b.dim() == 2 and a.dtype == b.dtype and a.dtype in _DT
    a, b = a.contiguous(), b.contiguous()
    M, K = (a.shape[1], a.shape[0]) if trans_a else (a.shape[0], a.shape[1])
    Kb, N = (b.shape[1], b.shape[0]) if trans_b else (b.shape[0], b.shape[1])
    assert K == Kb and K % 8 == 0
    out = torch.empty(M, N, dtype=a.dtype, device=a.device)
    am = A_COL if trans_a else A_ROW          # a^T stored [K][M]
    bm = B_ROW if trans_b else B_COL          # b^T stored [N][K] is K-contiguous
    lda = a.shape[1]
    ldb = b.shape[1]
    return gemm_raw(am, bm, a, lda, b, ldb, out, N, M, N, K, bias=bias, act=act)


# ----------------------------------------------------------------------------- conv
def _geo(N, H, W, C, OH, OW, KH, KW, sh, sw, ph, pw, dh, dw):
    return [N, H, W, C, OH, OW, KH, KW, sh, sw, ph, pw, dh, dw]


def supported(x, weight, groups):
    return (x.is_cuda and x.dtype in _DT and weight.dtype == x.dtype and groups == 1 and x.dim() == 4
            and x.shape[-1] % 8 == 0 and weight.shape[0] % 8 == 0 and _lib.native_available())


def conv_fwd(x, weight, stride, padding, dilation, bias=None, act=None):
    N, H, W, C = x.shape
    Co, Ci, KH, KW = weight.shape
    sh, sw = stride
    ph, pw = padding
    dh, dw = dilation
    OH = (H + 2 * ph - dh * (KH - 1) - 1) // sh + 1
    OW = (W + 2 * pw - dw * (KW - 1) - 1) // sw + 1
    wt = weight.permute(0, 2, 3, 1).contiguous()  # [Co][KH][KW][Ci] = B^T, K-contiguous
    out = torch.empty(N, OH, OW, Co, dtype=x.dtype, device=x.device)
    K = KH * KW * Ci
    gemm_raw(A_CONV, B_ROW, x.contiguous(), C, wt, K, out, Co, N * OH * OW, Co, K,
             bias=bias, act=act, conv=_geo(N, H, W, C, OH, OW, KH, KW, sh, sw, ph, pw, dh, dw))
    return out


def conv_bwd_data(dy, weight, x_shape, stride, padding, dilation):
    N, H, W, Ci = x_shape
    Co, _, KH, KW = weight.shape
    sh, sw = stride
    ph, pw = padding
    dh, dw = dilation
    _, OH, OW, _ = dy.shape
    dy = dy.contiguous()
    if (sh, sw) == (1, 1):
        # dX = conv(dY, flip(W)^T) with pad' = d*(K-1) - p, dilation d
        wt = weight.flip(2, 3).permute(1, 2, 3, 0).contiguous()  # [Ci][KH][KW][Co]
        dx = torch.empty(N, H, W, Ci, dtype=dy.dtype, device=dy.device)
        K = KH * KW * Co
        gemm_raw(A_CONV, B_ROW, dy, Co, wt, K, dx, Ci, N * H * W, Ci, K,
                 conv=_geo(N, OH, OW, Co, H, W, KH, KW, 1, 1, dh * (KH - 1) - ph, dw * (KW - 1) - pw, dh, dw))
        return dx
    if (dh, dw) != (1, 1):
        raise NotImplementedError("strided + dilated conv grad")
    dx = torch.zeros(N, H, W, Ci, dtype=dy.dtype, device=dy.device)
    for rh in range(sh):
        for rw in range(sw):
            hs = list(range(rh, H, sh))
            ws_ = list(range(rw, W, sw))
            if not hs or not ws_:
                continue
            # taps contributing to this output phase: kh = (rh + ph) mod sh + j*sh
            kh0, kw0 = (rh + ph) % sh, (rw + pw) % sw
            khs = list(range(kh0, KH, sh))
            kws = list(range(kw0, KW, sw))
            if not khs or not kws:
                continue
            bh, bw = (rh + ph - kh0) // sh, (rw + pw - kw0) // sw
            nh, nw = len(khs), len(kws)
            # phase output i' reads dY row i' + bh - j for tap j  ==  stride-1 conv with taps
            # reversed (t = nh-1-j) and pad = nh-1-bh
            # taps kh0, kh0 + sh, ... reversed: slices + flip (no host index tensor, so this
            # also runs inside a hipGraph capture)
            sub = weight[:, :, kh0::sh, :][:, :, :, kw0::sw].flip((2, 3))  # [Co][Ci][nh][nw]
            wt = sub.permute(1, 2, 3, 0).contiguous()  # [Ci][nh][nw][Co]
            PH, PW = len(hs), len(ws_)
            tmp = torch.empty(N, PH, PW, Ci, dtype=dy.dtype, device=dy.device)
            K = nh * nw * Co
            gemm_raw(A_CONV, B_ROW, dy, Co, wt, K, tmp, Ci, N * PH * PW, Ci, K,
                     conv=_geo(N, OH, OW, Co, PH, PW, nh, nw, 1, 1, nh - 1 - bh, nw - 1 - bw, 1, 1))
            dx[:, rh::sh, rw::sw, :] = tmp
    return dx


def conv_bwd_weight(dy, x, w_shape, stride, padding, dilation):
    Co, Ci, KH, KW = w_shape
    N, H, W, C = x.shape
    _, OH, OW, _ = dy.shape
    sh, sw = stride
    ph, pw = padding
    dh, dw = dilation
    M, Nn, K = Co, KH * KW * Ci, N * OH * OW
    dwt = torch.empty(Co, KH, KW, Ci, dtype=dy.dtype, device=dy.device)
    gemm_raw(A_COL, B_CONV, dy.contiguous(), Co, x.contiguous(), 0, dwt, Nn, M, Nn, K,
             conv=_geo(N, H, W, C, OH, OW, KH, KW, sh, sw, ph, pw, dh, dw))
    return dwt.permute(0, 3, 1, 2).contiguous()


class Conv2dNHWC(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, stride, padding, dilation):
        ctx.save_for_backward(x, weight)
        ctx.conf = (stride, padding, dilation, bias is not None)
        return conv_fwd(x, weight, stride, padding, dilation, bias=None if bias is None else bias.float())

    @staticmethod
    def backward(ctx, gy):
        x, weight = ctx.saved_tensors
        stride, padding, dilation, has_bias = ctx.conf
        gy = gy.contiguous()
        dx = conv_bwd_data(gy, weight, x.shape, stride, padding, dilation) if ctx.needs_input_grad[0] else None
        dw = conv_bwd_weight(gy, x, weight.shape, stride, padding, dilation) if ctx.needs_input_grad[1] else None
        db = gy.float().sum((0, 1, 2)).to(gy.dtype) if has_bias and ctx.needs_input_grad[2] else None
        return dx, dw, db, None, None, None


def conv2d_nhwc(x, weight, bias, stride, padding, dilation):
    return Conv2dNHWC.apply(x, weight, bias, tuple(stride), tuple(padding), tuple(dilation))


# ----------------------------------------------------------------------------------------------
# 256-row-tile kernels (csrc/kernels/gemm256.hip): glds-staged, 8 waves, 16x16x32 MFMA
# ----------------------------------------------------------------------------------------------
_ACT = {None: 0, "relu": 1, "gelu": 2}


def _L256():
    L = _L()
    if not getattr(L, "_g256_sig", False):
        P, I, LG = c_void_p, c_int, c_long
        L.pha_gemm256_nt.argtypes = [I, P, P, P, P, LG, LG, LG, LG, LG, LG, I, P, I, I, P]
        L.pha_gemm256_nt.restype = c_int
        L.pha_conv256_fwd.argtypes = [I, P, P, P, P] + [I] * 13 + [I, P, I, I, P, P, P, P, P, P, P, I, P, P]
        L.pha_gemm8p.argtypes = [I, P, P, P, P, LG, LG, LG, LG, LG, LG, I, I, I, P, I, P, P]
        L.pha_gemm8p.restype = c_int
        L.pha_gemm256_tn.argtypes = [I, P, P, P, P, LG, LG, LG, LG, LG, I, I, P, I, I, P]
        L.pha_gemm256_tn.restype = c_int
        L.pha_conv256_wgrad.argtypes = [I, P, P, P, P] + [I] * 13 + [I, P, I, I, P]
        L.pha_conv256_wgrad.restype = c_int
        L.pha_conv256_fwd.restype = c_int
        L.pha_conv256_fwd_f32out.argtypes = [I, P, P, P, P] + [I] * 13 + [I, P, I, I, P, P]
        L.pha_conv256_fwd_f32out.restype = c_int
        L.pha_conv256_fwd_grouped.argtypes = [I, P, P, P, P] + [I] * 15 + [LG, I, P, I, I, P, P]
        L.pha_conv256_fwd_grouped.restype = c_int
        L.pha_conv256_wgrad_grouped.argtypes = [I, P, P, P, P] + [I] * 15 + [P, I, I, P]
        L.pha_conv256_wgrad_grouped.restype = c_int
        L.pha_split3_f32.argtypes = [P, P, LG, LG, I, P]
        L.pha_split3_f32.restype = c_int
        L._g256_sig = True
    return L


def gemm8p(a, b, a_kouter=False, b_kouter=False, bias=None, act=None, out=None, splits=1):
    """C = op(A) @ op(B) on the 8-phase ping-pong MFMA kernel (gemm8p.hip).

    a: [M, K] (a_kouter=False) or [K, M]; b: B^T [N, K] (b_kouter=False) or B [K, N]. Row strides
    come from the tensors (unit inner stride); M, N, K and the strides % 8 == 0."""
    assert a.dtype in _DT and b.dtype == a.dtype and a.dim() == 2 and b.dim() == 2
    assert a.stride(1) == 1 and b.stride(1) == 1
    M, Ka = (a.shape[1], a.shape[0]) if a_kouter else (a.shape[0], a.shape[1])
    N, Kb = (b.shape[1], b.shape[0]) if b_kouter else (b.shape[0], b.shape[1])
    assert Ka == Kb, (a.shape, b.shape)
    c = out if out is not None else torch.empty(M, N, dtype=a.dtype, device=a.device)
    assert c.shape == (M, N) and c.stride(1) == 1
    if bias is not None:
        bias = bias.float().contiguous()
    ws = None
    if splits > 1:
        assert c.is_contiguous()
        ws = torch.empty(splits * M * N, dtype=torch.float32, device=a.device)
    rc = _L256().pha_gemm8p(_DT[a.dtype], _ptr(a), _ptr(b), _ptr(c), _ptr(bias), M, N, Ka, a.stride(0), b.stride(0),
                            c.stride(0), int(a_kouter), int(b_kouter), _ACT[act], _ptr(_zero_page(a.device)),
                            int(splits), _ptr(ws), c_void_p(torch.cuda.current_stream(a.device).cuda_stream))
    if rc != 0:
        raise RuntimeError(f"pha_gemm8p failed ({rc}) M={M} N={N} K={Ka}")
    return c


_tuned = {}
_CANDS = [(t, bk) for t in range(6) for bk in (32, 64)]


# Tile selection of the 256-row-tile conv / weight-gradient kernels is deterministic: a per-shape
# table measured once on MI355X and committed (tuning/conv256_gfx950.json, written by
# tools/tune_conv256.py), else the kernels' built-in heuristic. Timing on first use — the
# reference's opt-in kernel autotune (paddle.incubate.autotune.set_config({"kernel": {"enable":
# True}}), phi/kernels/autotune/) — runs only when enabled (or PHA_G256_AUTOTUNE=1), because a pick
# made by timing can differ between runs and between the ranks of one job.
TUNING_TABLE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuning",
                            "conv256_gfx950.json")
_table_cache = None
_timing_on = [None]


def _table():
    global _table_cache
    if _table_cache is None:
        try:
            with open(TUNING_TABLE) as f:
                _table_cache = json.load(f)
        except (OSError, ValueError):
            _table_cache = {}
    return _table_cache


def _kstr(key):
    return "|".join(str(k) for k in key)


def set_timing_autotune(on):
    """pick tiles by timing for shapes the table lacks (incubate.autotune kernel.enable)"""
    _timing_on[0] = bool(on)


def _timing():
    if _timing_on[0] is not None:
        return _timing_on[0]
    return os.environ.get("PHA_G256_AUTOTUNE", "0") == "1"


def _lookup(key):
    ch = _tuned.get(key)
    if ch is None:
        t = _table().get(_kstr(key))
        if t is not None:
            ch = tuple(t) if isinstance(t, list) else t
            _tuned[key] = ch
    return ch


def dump_tuning(path=None):
    """write every pick made so far (table + timed) as the JSON table"""
    out = dict(_table())
    for k, v in _tuned.items():
        out[_kstr(k)] = list(v) if isinstance(v, tuple) else v
    with open(path or TUNING_TABLE, "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)
    return len(out)


def _autotune(key, run):
    """(tile shape, BK) of the 256-row-tile kernels for this problem: the table's pick, else (with
    timing enabled, outside graph capture) the fastest candidate on the real operands, else the
    kernel heuristic (-1, 0)"""
    ch = _tuned.get(key) if _retune_conv[0] else _lookup(key)
    if ch is not None:
        return ch
    if not _timing() or torch.cuda.is_current_stream_capturing():
        return (-1, 0)
    best, best_t = (-1, 0), float("inf")
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for tile, bk in _CANDS:
        run(tile, bk)
        ev0.record()
        for _ in range(3):
            run(tile, bk)
        ev1.record()
        ev1.synchronize()
        t = ev0.elapsed_time(ev1)
        if t < best_t:
            best, best_t = (tile, bk), t
    _tuned[key] = best
    return best


def gemm256_nt(a, bt, bias=None, act=None, out=None):
    """C[M, N] = a[M, K] @ bt[N, K]^T (+ bias fp32[N]) (+ relu/gelu). K-contiguous operands."""
    assert a.dtype in _DT and bt.dtype == a.dtype and a.dim() == 2 and bt.dim() == 2 and a.shape[1] == bt.shape[1]
    assert a.stride(1) == 1 and bt.stride(1) == 1 and a.shape[1] % 8 == 0 and a.stride(0) % 8 == 0 and bt.stride(0) % 8 == 0
    M, K = a.shape
    N = bt.shape[0]
    c = out if out is not None else torch.empty((M, N), dtype=a.dtype, device=a.device)
    assert c.shape == (M, N) and c.stride(1) == 1
    if bias is not None:
        bias = bias.float().contiguous()
        assert bias.numel() == N
    L, z, st = _L256(), _ptr(_zero_page(a.device)), c_void_p(torch.cuda.current_stream(a.device).cuda_stream)

    def run(tile, bk):
        rc = L.pha_gemm256_nt(_DT[a.dtype], _ptr(a), _ptr(bt), _ptr(c), _ptr(bias), M, N, K, a.stride(0), bt.stride(0),
                              c.stride(0), _ACT[act], z, tile, bk, st)
        if rc != 0:
            raise RuntimeError(f"pha_gemm256_nt failed ({rc})")
    run(*_autotune(("gemm", a.dtype, M, N, K), run))
    return c


def conv256_fwd(x, w_okkc, stride, padding, dilation, bias=None, act=None, out=None, remap=None, bn_stats=False,
                bn_bwd=None, addend=None):
    """NHWC conv forward: x [N, H, W, C] (C % 8 == 0), w [Cout, KH, KW, C] -> y [N, OH, OW, Cout].

    ``remap = (oh0, ow0, osh, osw, OH, OW[, zero_rest])`` computes an OH x OW output and stores pixel
    (oh, ow) at (oh0 + oh*osh, ow0 + ow*osw) of ``out`` — one phase of a strided convolution's dgrad;
    ``zero_rest`` (with oh0 = ow0 = 0) also zero-fills the other pixels of each stride cell.
    ``bn_stats``: the epilogue also writes per-row-tile channel sums / sums of squares of y, attached
    as ``y._pha_bn_stats = (partials, rows, y._version)`` for the batch norm that consumes y.
    ``bn_bwd = (bn_x, mean, affine|None, partials, row0)``: y is the output gradient of that batch
    norm; the epilogue writes the BN backward's per-tile sums into partials from row row0 on and
    the call returns the number of rows written (with y in ``out``).
    ``addend``: a tensor shaped like y (not aliasing it) added in the epilogue after the activation
    — a dgrad that also receives the residual branch's gradient (no bn_stats / bn_bwd with it)."""
    assert x.dtype in _DT and w_okkc.dtype == x.dtype and x.is_contiguous() and w_okkc.is_contiguous()
    N, H, W, C = x.shape
    Co, KH, KW, Cw = w_okkc.shape
    assert C == Cw and C % 8 == 0
    sh, sw = stride
    ph, pw = padding
    dh, dw = dilation
    rm = None
    if remap is not None:
        assert out is not None and out.is_contiguous() and out.shape[0] == N and out.shape[3] == Co
        oh0, ow0, osh, osw, OH, OW = remap[:6]
        zr = int(len(remap) > 6 and bool(remap[6]))
        assert oh0 + (OH - 1) * osh < out.shape[1] and ow0 + (OW - 1) * osw < out.shape[2]
        assert not zr or (oh0 == ow0 == 0 and OH * osh >= out.shape[1] and OW * osw >= out.shape[2] and Co % 8 == 0)
        rm = (c_int * 9)(out.shape[1], out.shape[2], oh0, ow0, osh, osw, OH, OW, zr)
        y = out
    else:
        OH = (H + 2 * ph - dh * (KH - 1) - 1) // sh + 1
        OW = (W + 2 * pw - dw * (KW - 1) - 1) // sw + 1
        y = out if out is not None else torch.empty((N, OH, OW, Co), dtype=x.dtype, device=x.device)
        assert y.shape == (N, OH, OW, Co) and y.is_contiguous()
    if bias is not None:
        bias = bias.float().contiguous()
    L, z, st = _L256(), _ptr(_zero_page(x.device)), c_void_p(torch.cuda.current_stream(x.device).cuda_stream)
    part, rows = None, c_int(0)
    if bn_stats and rm is None and bn_bwd is None:
        part = torch.empty(-(-(N * OH * OW) // 128) * 2 * Co, dtype=torch.float32, device=x.device)
    bx, bmean, baff, bpart, brow0 = bn_bwd if bn_bwd is not None else (None, None, None, None, 0)
    if addend is not None:
        assert part is None and bpart is None and (rm is None or rm[8] == 0)
        assert addend.shape == y.shape and addend.dtype == y.dtype and addend.is_contiguous()
        assert addend.data_ptr() != y.data_ptr()

    def run(tile, bk):
        rc = L.pha_conv256_fwd(_DT[x.dtype], _ptr(x), _ptr(w_okkc), _ptr(y), _ptr(bias), N, H, W, C, Co, KH, KW,
                               sh, sw, ph, pw, dh, dw, _ACT[act], z, tile, bk, rm, _ptr(part),
                               byref(rows) if (part is not None or bpart is not None) else None,
                               _ptr(bx), _ptr(bmean), _ptr(baff), _ptr(bpart), int(brow0), _ptr(addend), st)
        if rc != 0:
            raise RuntimeError(f"pha_conv256_fwd failed ({rc})")
    run(*_autotune(("conv", x.dtype, N, H, W, C, Co, KH, KW, sh, sw, ph, pw, dh, dw, OH, OW), run))
    if part is not None:
        y._pha_bn_stats = (part, rows.value, y._version)
    if bpart is not None:
        return y, rows.value
    return y


def conv256_dgrad(dy, w, x_shape, stride, padding, dilation, bn_src=None, addend=None, f32=False):
    """dx [N, H, W, Ci] of an NHWC conv from dy [N, OH, OW, Co] and w [Co, Ci, KH, KW], on the forward
    kernel: stride 1 is the conv of dy with the flipped, transposed filter (pad' = d*(K-1) - p);
    stride s splits dx into s*s phases, each a stride-1 conv over the taps that reach it, stored
    in place through the kernel's output remap (no scatter copy).

    ``bn_src = (bn_x, mean, affine|None, token)``: dx is the output gradient of that batch norm;
    its backward sums are reduced in the epilogue and attached as ``dx._pha_bn_bwd``.
    ``addend``: another gradient of x (the residual branch's), summed into dx — in the stride-1
    epilogue, else by one add after the phases.
    ``f32``: fp32 dy / w / dx through the three-term bf16 split (``split3``): dy's channels
    [hi, hi, lo] against filters [hi, lo, hi] along Co, fp32 epilogue stores."""
    N, H, W, Ci = x_shape
    Co, _, KH, KW = w.shape
    sh, sw = stride
    ph, pw = padding
    dh, dw = dilation
    _, OH, OW, _ = dy.shape
    dy = dy.contiguous()
    if f32:
        return _dgrad_f32(dy, w, x_shape, stride, padding, dilation)
    assert addend is None or (tuple(addend.shape) == (N, H, W, Ci) and addend.dtype == dy.dtype), x_shape
    if addend is not None:
        addend = addend.contiguous()
        bn_src = None   # the BN-backward epilogue sums would miss the addend
    bn = None
    if bn_src is not None and Ci % 8 == 0 and bn_src[0].shape == (N, H, W, Ci) and bn_src[0].is_contiguous():
        # rows: every launch below writes <= ceil(rows / 128) partial rows
        bn = [bn_src, torch.empty((-(-(N * H * W) // 128) + 4 * sh * sw) * 2 * Ci, dtype=torch.float32,
                                  device=dy.device), 0]

    def _bn(): return None if bn is None else (bn[0][0], bn[0][1], bn[0][2], bn[1], bn[2])

    def _run(*args, **kw):
        r = conv256_fwd(*args, bn_bwd=_bn(), **kw)
        if bn is not None:
            bn[2] += r[1]
            return r[0]
        return r

    def _done(dx):
        if bn is not None:
            dx._pha_bn_bwd = (bn[1], bn[2], bn[0][3], dx._version)
        return dx
    if (sh, sw) == (1, 1):
        wt = _wlayout(w, "dgrad", lambda t: _flip_hw(t).permute(1, 2, 3, 0).contiguous())   # [Ci][KH][KW][Co]
        dx = torch.empty(N, H, W, Ci, dtype=dy.dtype, device=dy.device)
        return _done(_run(dy, wt, (1, 1), (dh * (KH - 1) - ph, dw * (KW - 1) - pw), (dh, dw), out=dx,
                          remap=(0, 0, 1, 1, H, W), addend=addend))
    if addend is not None:
        return conv256_dgrad(dy, w, x_shape, stride, padding, dilation).add_(addend)
    if (dh, dw) != (1, 1):
        raise NotImplementedError("strided + dilated conv dgrad")
    phases = []
    for rh in range(sh):
        for rw in range(sw):
            PH, PW = len(range(rh, H, sh)), len(range(rw, W, sw))
            kh0, kw0 = (rh + ph) % sh, (rw + pw) % sw
            khs, kws = list(range(kh0, KH, sh)), list(range(kw0, KW, sw))
            phases.append((rh, rw, PH, PW, khs, kws, kh0, kw0))
    live = [p for p in phases if p[2] and p[3] and p[4] and p[5]]
    # only phase (0, 0) reached (1x1 stride-s filters): its kernel zero-fills the stride cells
    zero_rest = len(live) == 1 and live[0][:2] == (0, 0) and live[0][2] * sh >= H and live[0][3] * sw >= W \
        and Ci % 8 == 0
    full = len(live) == len(phases) or zero_rest
    dx = (torch.empty if full else torch.zeros)(N, H, W, Ci, dtype=dy.dtype, device=dy.device)
    if bn is not None and not full:
        bn = None   # rows of never-written (zero) phases would miss the epilogue sums: BN reduces itself
    for rh, rw, PH, PW, khs, kws, kh0, kw0 in live:
        # output row i of the phase (input row rh + i*sh) receives dy row i + bh - j through tap
        # khs[j]: a stride-1 conv over the reversed taps with top padding nh - 1 - bh
        bh, bw = (rh + ph - kh0) // sh, (rw + pw - kw0) // sw
        nh, nw = len(khs), len(kws)
        wt = _wlayout(w, ("phase", rh, rw, sh, sw, ph, pw), lambda t, kh0=kh0, kw0=kw0:   # reversed taps
                      t[:, :, kh0::sh, :][:, :, :, kw0::sw].flip((2, 3)).permute(1, 2, 3, 0).contiguous())   # [Ci][nh][nw][Co]
        _run(dy, wt, (1, 1), (nh - 1 - bh, nw - 1 - bw), (1, 1), out=dx,
             remap=(rh, rw, sh, sw, PH, PW, zero_rest))
    return _done(dx)


_wlayouts = {}


# ----------------------------------------------------------------------------------------------
# fp32 convolutions on the bf16 MFMA kernels: x = xh + xl, w = wh + wl (bf16 hi / lo parts), and
# x.w ~= xh.wh + xh.wl + xl.wh — the lo.lo term is below fp32 rounding of most products (2^-16
# relative). The three products are ONE implicit GEMM over concatenated channels [xh, xh, xl] x
# [wh, wl, wh] with an fp32 epilogue, so Paddle's default-dtype convolutions run on the matrix
# cores at ~5x the fp32 MFMA rate instead of on MIOpen (reference: phi/kernels/gpudnn/
# conv_kernel.cu, cuDNN's fp32 / TF32 paths).
# ----------------------------------------------------------------------------------------------
def split3(t, dim, order="hhl"):
    """fp32 t -> bf16 parts concatenated along ``dim`` in ``order`` (h = hi, l = lo); one pass of
    csrc/kernels/split.hip on the GPU"""
    assert len(order) == 3 and set(order) <= {"h", "l"}, f"split3 takes three parts, got {order!r}"
    dim = dim % t.dim()
    inner = t[(0,) * dim].numel() if t.numel() else 0
    if (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() and inner and inner % 8 == 0
            and t.data_ptr() % 16 == 0 and _lib.native_available()):
        shape = list(t.shape)
        shape[dim] *= 3
        out = torch.empty(shape, dtype=torch.bfloat16, device=t.device)
        mask = sum(1 << i for i, c in enumerate(order) if c == "l")
        rc = _L256().pha_split3_f32(_ptr(t), _ptr(out), t.numel() // inner, inner, mask,
                                     c_void_p(torch.cuda.current_stream(t.device).cuda_stream))
        if rc == 0:
            return out
    hi = t.to(torch.bfloat16)
    fin = torch.isfinite(t)
    # finite past the bf16 range: truncate instead of rounding to inf (no host sync: graph-capturable)
    over = fin & ~torch.isfinite(hi)
    hi = torch.where(over, (t.contiguous().view(torch.int32) >> 16).to(torch.int16).view(torch.bfloat16), hi)
    lo = torch.where(fin, t - hi.float(), torch.zeros_like(t)).to(torch.bfloat16)
    return torch.cat([hi if c == "h" else lo for c in order], dim)


def conv256_fwd_f32(x3, w3, stride, padding, dilation, bias=None, act=None, out=None, remap=None):
    """NHWC conv with an fp32 output from pre-split bf16 operands: x3 [N, H, W, 3C] ([hi, hi, lo]),
    w3 [Co, KH, KW, 3C] ([hi, lo, hi])"""
    assert x3.dtype == torch.bfloat16 and w3.dtype == x3.dtype and x3.is_contiguous() and w3.is_contiguous()
    N, H, W, C = x3.shape
    Co, KH, KW, Cw = w3.shape
    assert C == Cw and C % 8 == 0
    sh, sw = stride
    ph, pw = padding
    dh, dw = dilation
    rm = None
    if remap is not None:
        assert out is not None and out.is_contiguous() and out.dtype == torch.float32
        oh0, ow0, osh, osw, OH, OW = remap[:6]
        zr = int(len(remap) > 6 and bool(remap[6]))
        rm = (c_int * 9)(out.shape[1], out.shape[2], oh0, ow0, osh, osw, OH, OW, zr)
        y = out
    else:
        OH = (H + 2 * ph - dh * (KH - 1) - 1) // sh + 1
        OW = (W + 2 * pw - dw * (KW - 1) - 1) // sw + 1
        y = out if out is not None else torch.empty((N, OH, OW, Co), dtype=torch.float32, device=x3.device)
        assert y.shape == (N, OH, OW, Co) and y.is_contiguous() and y.dtype == torch.float32
    if bias is not None:
        bias = bias.float().contiguous()
    L, z, st = _L256(), _ptr(_zero_page(x3.device)), c_void_p(torch.cuda.current_stream(x3.device).cuda_stream)
    rc = L.pha_conv256_fwd_f32out(_DT[x3.dtype], _ptr(x3), _ptr(w3), _ptr(y), _ptr(bias), N, H, W, C, Co, KH, KW,
                                  sh, sw, ph, pw, dh, dw, _ACT[act], z, -1, 0, rm, st)
    if rc != 0:
        raise RuntimeError(f"pha_conv256_fwd_f32out failed ({rc})")
    return y


def _dgrad_f32(dy, w, x_shape, stride, padding, dilation):
    """fp32 dx of an NHWC conv (see conv256_dgrad): dy split along Co as [hi, hi, lo], the dgrad
    filter layouts (Co last) split as [hi, lo, hi]"""
    N, H, W, Ci = x_shape
    Co, _, KH, KW = w.shape
    sh, sw = stride
    ph, pw = padding
    dh, dw = dilation
    dy3 = split3(dy, 3, "hhl")
    if (sh, sw) == (1, 1):
        wt = _wlayout(w, "dgrad_f32", lambda t: split3(t.flip(2, 3).permute(1, 2, 3, 0).contiguous(), 3, "hlh"))
        dx = torch.empty(N, H, W, Ci, dtype=torch.float32, device=dy.device)
        return conv256_fwd_f32(dy3, wt, (1, 1), (dh * (KH - 1) - ph, dw * (KW - 1) - pw), (dh, dw), out=dx,
                               remap=(0, 0, 1, 1, H, W))
    if (dh, dw) != (1, 1):
        raise NotImplementedError("strided + dilated conv dgrad")
    phases = []
    for rh in range(sh):
        for rw in range(sw):
            PH, PW = len(range(rh, H, sh)), len(range(rw, W, sw))
            kh0, kw0 = (rh + ph) % sh, (rw + pw) % sw
            khs, kws = list(range(kh0, KH, sh)), list(range(kw0, KW, sw))
            phases.append((rh, rw, PH, PW, khs, kws, kh0, kw0))
    live = [p for p in phases if p[2] and p[3] and p[4] and p[5]]
    zero_rest = len(live) == 1 and live[0][:2] == (0, 0) and live[0][2] * sh >= H and live[0][3] * sw >= W
    full = len(live) == len(phases) or zero_rest
    dx = (torch.empty if full else torch.zeros)(N, H, W, Ci, dtype=torch.float32, device=dy.device)
    for rh, rw, PH, PW, khs, kws, kh0, kw0 in live:
        bh, bw = (rh + ph - kh0) // sh, (rw + pw - kw0) // sw
        nh, nw = len(khs), len(kws)
        wt = _wlayout(w, ("phase_f32", rh, rw, sh, sw, ph, pw), lambda t, kh0=kh0, kw0=kw0: split3(
            t[:, :, kh0::sh, :][:, :, :, kw0::sw].flip((2, 3)).permute(1, 2, 3, 0).contiguous(), 3, "hlh"))
        conv256_fwd_f32(dy3, wt, (1, 1), (nh - 1 - bh, nw - 1 - bw), (1, 1), out=dx,
                        remap=(rh, rw, sh, sw, PH, PW, zero_rest))
    return dx


class Conv2dNHWC256F32(torch.autograd.Function):
    """fp32 NHWC conv2d: forward, dgrad and wgrad as three-term bf16 MFMA products (split3)"""

    @staticmethod
    def forward(ctx, x, weight, bias, stride, padding, dilation):
        ctx.save_for_backward(x)
        ctx.weight = weight
        ctx.conf = (stride, padding, dilation, bias is not None)
        w3 = _wlayout(weight, "fwd_f32", lambda t: split3(t.permute(0, 2, 3, 1).contiguous(), 3, "hlh"))
        return conv256_fwd_f32(split3(x.contiguous(), 3, "hhl"), w3, stride, padding, dilation, bias=bias)

    @staticmethod
    def backward(ctx, gy):
        x, = ctx.saved_tensors
        weight = ctx.weight
        stride, padding, dilation, has_bias = ctx.conf
        gy = gy.contiguous().float()
        dx = conv256_dgrad(gy, weight, x.shape, stride, padding, dilation, f32=True) \
            if ctx.needs_input_grad[0] else None
        dw = None
        if ctx.needs_input_grad[1]:
            # the reduction runs over pixels: stack the split along the batch ([dy_h; dy_h; dy_l] x
            # [x_h; x_l; x_h]) and let the weight-gradient GEMM sum the three terms in fp32
            dw = conv256_wgrad(split3(gy, 0, "hhl"), split3(x.contiguous(), 0, "hlh"), weight.shape, stride, padding,
                               dilation, out_dtype=torch.float32)
        db = gy.sum((0, 1, 2)) if has_bias and ctx.needs_input_grad[2] else None
        return dx, dw, db, None, None, None


# ----------------------------------------------------------------------------------------------
# grouped convolutions (ResNeXt's 3x3 group convs) as ONE grouped implicit GEMM per pass: blockIdx.y
# = group, each group's GEMM over its own input channels / filter rows / output columns
# (gemm256.hip ConvGeo cs / ga / gb / gc). Groups narrower than 8 input channels are merged in
# pairs / quads with block-diagonal zero filters (a few x the FLOPs of those small convs, on the
# matrix cores instead of the VALU kernels).
# ----------------------------------------------------------------------------------------------
def _gfwd(x, w_g, groups, cig, cog, stride, padding, dilation, out=None, remap=None, bias=None):
    """x [N, H, W, groups*cig], w_g [groups*cog, KH, KW, cig] -> y [N, OH, OW, groups*cog]"""
    N, H, W, C = x.shape
    _, KH, KW, _ = w_g.shape
    sh, sw = stride
    ph, pw = padding
    dh, dw = dilation
    rm = None
    if remap is not None:
        oh0, ow0, osh, osw, OH, OW = remap[:6]
        zr = int(len(remap) > 6 and bool(remap[6]))
        rm = (c_int * 9)(out.shape[1], out.shape[2], oh0, ow0, osh, osw, OH, OW, zr)
        y = out
    else:
        OH = (H + 2 * ph - dh * (KH - 1) - 1) // sh + 1
        OW = (W + 2 * pw - dw * (KW - 1) - 1) // sw + 1
        y = out if out is not None else torch.empty((N, OH, OW, groups * cog), dtype=x.dtype, device=x.device)
    L, z, st = _L256(), _ptr(_zero_page(x.device)), c_void_p(torch.cuda.current_stream(x.device).cuda_stream)
    rc = L.pha_conv256_fwd_grouped(_DT[x.dtype], _ptr(x), _ptr(w_g), _ptr(y), _ptr(bias), N, H, W, cig, cog, groups,
                                   KH, KW, sh, sw, ph, pw, dh, dw, _ACT[None], y.shape[-1], 0, z, -1, 0, rm, st)
    if rc != 0:
        raise RuntimeError(f"pha_conv256_fwd_grouped failed ({rc})")
    return y


def _merge_groups(w, groups, m):
    """[Co, cig, KH, KW] grouped filters -> [Co, cig*m, KH, KW] for groups / m groups, each merged
    group's filter block-diagonal (zeros between the original groups)"""
    Co, cig, KH, KW = w.shape
    cog = Co // groups
    wg = w.reshape(groups // m, m, cog, cig, KH, KW)
    out = w.new_zeros(groups // m, m, cog, m, cig, KH, KW)
    for i in range(m):
        out[:, i, :, i] = wg[:, i]
    return out.reshape(Co, m * cig, KH, KW)


class GroupedConv2dNHWC256(torch.autograd.Function):
    """grouped NHWC conv2d: forward, dgrad (flipped / phase filters, grouped) and wgrad (grouped TN
    with per-group split-K slabs) on the 256-tile MFMA kernels"""

    @staticmethod
    def forward(ctx, x, weight, bias, stride, padding, dilation, groups):
        Co, cig, KH, KW = weight.shape
        cog = Co // groups
        ctx.save_for_backward(x)
        ctx.weight, ctx.conf = weight, (stride, padding, dilation, groups, bias is not None)
        wg = _wlayout(weight, ("gfwd", groups), lambda t: t.permute(0, 2, 3, 1).contiguous())
        y = _gfwd(x.contiguous(), wg, groups, cig, cog, stride, padding, dilation)
        return y.add_(bias.to(y.dtype)) if bias is not None else y

    @staticmethod
    def backward(ctx, gy):
        x, = ctx.saved_tensors
        w = ctx.weight
        stride, padding, dilation, groups, has_bias = ctx.conf
        Co, cig, KH, KW = w.shape
        cog = Co // groups
        gy = gy.contiguous()
        N, H, W, C = x.shape
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = _gdgrad(gy, w, (N, H, W, C), stride, padding, dilation, groups)
        if ctx.needs_input_grad[1]:
            dw = _gwgrad(gy, x.contiguous(), w.shape, stride, padding, dilation, groups)
        if has_bias and ctx.needs_input_grad[2]:
            db = gy.float().sum((0, 1, 2)).to(gy.dtype)
        return dx, dw, db, None, None, None, None


def _gdgrad(dy, w, x_shape, stride, padding, dilation, groups):
    N, H, W, C = x_shape
    Co, cig, KH, KW = w.shape
    cog = Co // groups
    sh, sw = stride
    ph, pw = padding
    dh, dw = dilation

    def gt(t):   # [Co, cig, kh, kw] (taps already selected / flipped) -> [groups*cig, kh, kw, cog]
        g_, kh, kw = groups, t.shape[2], t.shape[3]
        return t.reshape(g_, cog, cig, kh, kw).permute(0, 2, 3, 4, 1).reshape(g_ * cig, kh, kw, cog).contiguous()
    if (sh, sw) == (1, 1):
        wt = _wlayout(w, ("gdgrad", groups), lambda t: gt(t.flip(2, 3)))
        dx = torch.empty(N, H, W, C, dtype=dy.dtype, device=dy.device)
        return _gfwd(dy, wt, groups, cog, cig, (1, 1), (dh * (KH - 1) - ph, dw * (KW - 1) - pw), (dh, dw), out=dx,
                     remap=(0, 0, 1, 1, H, W))
    if (dh, dw) != (1, 1):
        raise NotImplementedError("strided + dilated grouped conv dgrad")
    phases = []
    for rh in range(sh):
        for rw in range(sw):
            PH, PW = len(range(rh, H, sh)), len(range(rw, W, sw))
            kh0, kw0 = (rh + ph) % sh, (rw + pw) % sw
            khs, kws = list(range(kh0, KH, sh)), list(range(kw0, KW, sw))
            phases.append((rh, rw, PH, PW, khs, kws, kh0, kw0))
    live = [p for p in phases if p[2] and p[3] and p[4] and p[5]]
    zero_rest = len(live) == 1 and live[0][:2] == (0, 0) and live[0][2] * sh >= H and live[0][3] * sw >= W \
        and cig % 8 == 0
    full = len(live) == len(phases) or zero_rest
    dx = (torch.empty if full else torch.zeros)(N, H, W, C, dtype=dy.dtype, device=dy.device)
    for rh, rw, PH, PW, khs, kws, kh0, kw0 in live:
        bh, bw = (rh + ph - kh0) // sh, (rw + pw - kw0) // sw
        nh, nw = len(khs), len(kws)
        wt = _wlayout(w, ("gphase", groups, rh, rw, sh, sw, ph, pw), lambda t, kh0=kh0, kw0=kw0:
                      gt(t[:, :, kh0::sh, :][:, :, :, kw0::sw].flip((2, 3))))
        _gfwd(dy, wt, groups, cog, cig, (1, 1), (nh - 1 - bh, nw - 1 - bw), (1, 1), out=dx,
              remap=(rh, rw, sh, sw, PH, PW, zero_rest))
    return dx


def _gwgrad(dy, x, w_shape, stride, padding, dilation, groups):
    Co, cig, KH, KW = w_shape
    cog = Co // groups
    N, H, W, C = x.shape
    _, OH, OW, _ = dy.shape
    sh, sw = stride
    ph, pw = padding
    dh, dw = dilation
    out = torch.empty(Co, cig, KH, KW, dtype=dy.dtype, device=dy.device)
    M, Nn, K = cog, KH * KW * cig, N * OH * OW
    sp = max(1, min(32, K // 32 // 8, -(-2 * _num_cus(dy.device) // max(1, groups * -(-M // 128) * -(-Nn // 128)))))
    ws = torch.empty(groups * sp * M * Nn, dtype=torch.float32, device=dy.device)
    L, z, st = _L256(), _ptr(_zero_page(x.device)), c_void_p(torch.cuda.current_stream(x.device).cuda_stream)
    rc = L.pha_conv256_wgrad_grouped(_DT[dy.dtype], _ptr(dy), _ptr(x), _ptr(out), _ptr(ws), N, H, W, cig, cog, groups,
                                     KH, KW, sh, sw, ph, pw, dh, dw, 0, z, -1, sp, st)
    if rc != 0:
        raise RuntimeError(f"pha_conv256_wgrad_grouped failed ({rc})")
    return out


def grouped_ok(x, w, groups):
    """bf16 / fp16 grouped convs the grouped implicit GEMM takes (after merging narrow groups)"""
    import os
    if os.environ.get("PHA_GCONV_MFMA", "1") == "0" or groups <= 1 or w.dtype != x.dtype \
            or x.dtype not in (torch.bfloat16, torch.float16) or not x.is_cuda:
        return False
    Co, cig = w.shape[0], w.shape[1]
    if Co % groups or cig * groups != x.shape[-1]:
        return False
    cog = Co // groups
    m = _merge_factor(cig, cog, groups)
    return m is not None and cig * m >= 8


def _merge_factor(cig, cog, groups):
    """smallest m (dividing groups) with cig*m and cog*m multiples of 8"""
    for m in (1, 2, 4, 8):
        if groups % m == 0 and (cig * m) % 8 == 0 and (cog * m) % 8 == 0:
            return m
    return None


def conv2d_nhwc256_grouped(x, weight, bias, stride, padding, dilation, groups):
    Co, cig = weight.shape[0], weight.shape[1]
    m = _merge_factor(cig, Co // groups, groups)
    if m > 1:   # narrow groups: merge m of them with block-diagonal filters (autograd through the merge)
        weight = _merge_groups(weight, groups, m)
        groups //= m
    return GroupedConv2dNHWC256.apply(x, weight, bias, tuple(stride), tuple(padding), tuple(dilation), groups)


def conv2d_nhwc256_f32(x, weight, bias, stride, padding, dilation):
    return Conv2dNHWC256F32.apply(x, weight, bias, tuple(stride), tuple(padding), tuple(dilation))


def _flip_hw(t):
    """the filter's spatial flip (a no-op, and no kernel, for 1x1 filters)"""
    return t if t.shape[2] == 1 and t.shape[3] == 1 else t.flip(2, 3)


def _wlayout(w, kind, make):
    """filter re-layouts (forward [Co][KH][KW][Ci], flipped dgrad filters, dgrad phase filters)
    cached per parameter version: computed once per optimizer step, not once per call. One entry
    per (parameter, kind): a new version replaces (and frees) the stale copy before the new one is
    made, so the cache holds at most one re-layout of every weight (keying by version kept up to
    512 stale copies alive: +50 GB on GPT-3 13B)."""
    import weakref
    key = (w.data_ptr(), tuple(w.shape), w.dtype, kind)
    hit = _wlayouts.get(key)
    if hit is not None and hit[0]() is w and hit[2] == w._version:
        return hit[1]
    _wlayouts.pop(key, None)
    hit = None
    if len(_wlayouts) > 4096:
        _wlayouts.clear()
    with torch.no_grad():
        v = make(w.detach())
    _wlayouts[key] = (weakref.ref(w), v, w._version)
    return v


_TN_CANDS = [(256, 256), (256, 128), (128, 256), (128, 128), (64, 256), (256, 64), (128, 64), (64, 128)]


def _tn_splits(M, N, K, tile, dev):
    bm, bn = _TN_CANDS[tile]
    tiles = -(-M // bm) * -(-N // bn)
    kblocks = -(-K // 32)
    return max(1, min(kblocks // 8, -(-2 * _num_cus(dev) // tiles), kblocks))


def _tn_tiles(M, N):
    """candidate tiles whose padding waste stays under 2x"""
    out = []
    for t, (bm, bn) in enumerate(_TN_CANDS):
        pad = (-(-M // bm) * bm) * (-(-N // bn) * bn)
        if pad <= 2 * M * N or (bm == 64 and bn == 128):
            out.append(t)
    return out


def _tn_ws(sp, M, N, dev):
    """fp32 split-K workspace: the partials plus the first-level sums of 16 (splits > 32)"""
    return torch.empty((sp + (-(-sp // 16) if sp > 32 else 0)) * M * N, dtype=torch.float32, device=dev)


_TN_SPLIT_CANDS = (1, 2, 4, 8, 16, 24, 32, 48, 64, 96, 128, 192, 256, 384, 512)
_retune_tn = [False]   # tools/tune_conv256.py --retune-tn: time TN launches even where the table has a pick
_retune_conv = [False]   # tools/tune_conv256.py --retune-all: the same for the forward / dgrad launches


def _run_tn(key, M, N, K, dev, call):
    """the (tile, split-K factor) of a TN launch: the table's pick — [tile, splits], or a bare tile
    with the formula's splits — else, with timing enabled, the fastest of every candidate tile x
    split factor (the formula's two rounds of work items is 1.1-1.6x off the best on ResNet-50's
    small-output wgrads, profiles/wgrad_split_r5/), else the fewest padded tiles with the formula's
    splits; call(tile, splits, ws) launches it"""
    ch = _tuned.get(key) if _retune_tn[0] else _lookup(key)
    if ch is None:
        tiles = _tn_tiles(M, N)
        if not _timing() or torch.cuda.is_current_stream_capturing():
            # fewest tiles (least MFMA padding), larger tiles first on ties
            ch = min(tiles, key=lambda t: -(-M // _TN_CANDS[t][0]) * -(-N // _TN_CANDS[t][1]))
        else:
            best_t = float("inf")
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            kb = -(-K // 32)
            for t in tiles:
                cands = sorted({s for s in _TN_SPLIT_CANDS if s <= max(1, kb // 4)} | {_tn_splits(M, N, K, t, dev)})
                for sp in cands:
                    ws = _tn_ws(sp, M, N, dev)
                    call(t, sp, ws)
                    ev0.record()
                    for _ in range(5):
                        call(t, sp, ws)
                    ev1.record()
                    ev1.synchronize()
                    el = ev0.elapsed_time(ev1)
                    if el < best_t:
                        best_t, ch = el, (t, sp)
            _tuned[key] = ch
    if isinstance(ch, tuple):
        t, sp = ch
    else:
        t, sp = ch, _tn_splits(M, N, K, ch, dev)
    call(t, sp, _tn_ws(sp, M, N, dev))


def gemm256_tn(a, b, out=None, out_dtype=None, accumulate=False):
    """C[M, N] = a[K, M]^T @ b[K, N] — the weight-gradient product (X^T dY) with both operands
    K-outer as they come out of the forward; fp32 split-K partials, result in ``out_dtype``
    (default a.dtype; torch.float32 for master-weight gradients) or added into ``out``."""
    assert a.dtype in _DT and b.dtype == a.dtype and a.dim() == 2 and b.dim() == 2 and a.shape[0] == b.shape[0]
    assert a.stride(1) == 1 and b.stride(1) == 1
    K, M = a.shape
    N = b.shape[1]
    od = out.dtype if out is not None else (out_dtype or a.dtype)
    if out is None:
        out = torch.empty(M, N, dtype=od, device=a.device)
        accumulate = False
    assert out.shape == (M, N) and out.is_contiguous() and od in (a.dtype, torch.float32)
    L, z, st = _L256(), _ptr(_zero_page(a.device)), c_void_p(torch.cuda.current_stream(a.device).cuda_stream)

    tgt = {"out": out, "acc": int(accumulate)}

    def call(tile, splits, ws):
        rc = L.pha_gemm256_tn(_DT[a.dtype], _ptr(a), _ptr(b), _ptr(tgt["out"]), _ptr(ws), M, N, K, a.stride(0),
                              b.stride(0), int(od == torch.float32), tgt["acc"], z, tile, splits, st)
        if rc != 0:
            raise RuntimeError(f"pha_gemm256_tn failed ({rc})")
    if accumulate and ("tn", a.dtype, M, N, K) not in _tuned:
        # autotuning launches the product several times: tune on a scratch output first
        tgt.update(out=torch.empty_like(out), acc=0)
        _run_tn(("tn", a.dtype, M, N, K), M, N, K, a.device, call)
        tgt.update(out=out, acc=1)
    _run_tn(("tn", a.dtype, M, N, K), M, N, K, a.device, call)
    return out


def conv256_wgrad(dy, x, w_shape, stride, padding, dilation, out_dtype=None):
    """dw [Co, Ci, KH, KW] of an NHWC conv: dy [N, OH, OW, Co], x [N, H, W, Ci] (Ci, Co % 8 == 0)."""
    Co, Ci, KH, KW = w_shape
    N, H, W, C = x.shape
    assert C == Ci and C % 8 == 0 and Co % 8 == 0 and dy.shape[-1] == Co
    dy, x = dy.contiguous(), x.contiguous()
    _, OH, OW, _ = dy.shape
    sh, sw = stride
    ph, pw = padding
    dh, dw = dilation
    od = out_dtype or dy.dtype
    out = torch.empty(Co, Ci, KH, KW, dtype=od, device=dy.device)
    M, Nn, K = Co, KH * KW * Ci, N * OH * OW
    L, z, st = _L256(), _ptr(_zero_page(x.device)), c_void_p(torch.cuda.current_stream(x.device).cuda_stream)

    def call(tile, splits, ws):
        rc = L.pha_conv256_wgrad(_DT[dy.dtype], _ptr(dy), _ptr(x), _ptr(out), _ptr(ws), N, H, W, C, Co, KH, KW,
                                 sh, sw, ph, pw, dh, dw, int(od == torch.float32), z, tile, splits, st)
        if rc != 0:
            raise RuntimeError(f"pha_conv256_wgrad failed ({rc})")
    _run_tn(("wgrad", dy.dtype, N, H, W, C, Co, KH, KW, sh, sw, ph, pw, dh, dw), M, Nn, K, x.device, call)
    return out


def _bn_stats_on():
    import os
    return os.environ.get("PHA_CONV_BN_STATS", "1") != "0"


def _bn_bwd_on():
    """dgrad epilogue reduces the preceding batch norm's backward sums (PHA_CONV_BN_BWD=1: on).
    Off by default: measured on ResNet-50 (batch 256) the extra bn_x reads at the end of every dgrad
    tile cost more than the skipped reduction pass saves (7.74k img/s vs 7.94k with it off, same box)."""
    import os
    return _bn_stats_on() and os.environ.get("PHA_CONV_BN_BWD", "0") == "1"


def res_route_begin(x, kind="bn"):
    """Residual-gradient route for a residual block whose input ``x`` (torch tensor) feeds exactly
    two ops: the block's first convolution and (kind "bn") as ``residual`` the fused BN-add-ReLU that
    ends the block, or (kind "conv") the downsample shortcut's convolution. Autograd would add the
    two gradients of x in a separate pass; with the route, the other consumer's backward hands its
    gradient of x over and the first convolution's dgrad epilogue adds it (one fewer read + write of
    the activation gradient per block). Returns the route token (or None when not applicable); call
    ``res_route_end`` after the block's forward."""
    import os
    if os.environ.get("PHA_RES_ROUTE", "1") == "0" or not torch.is_grad_enabled() or not x.requires_grad \
            or not x.is_cuda or x.dtype not in _DT or x.dim() != 4:
        return None
    if kind == "conv" and os.environ.get("PHA_RES_ROUTE_CONV", "1") == "0":
        return None
    route = {"armed": False, "kind": kind}
    x._pha_res_route = route
    return route


def res_route_end(x, route):
    if route is not None:
        try:
            del x._pha_res_route
        except AttributeError:
            pass
        if route.get("armed") and not route.get("sink"):
            route["armed"] = False   # no fused BN took the residual: nothing is handed over


class Conv2dNHWC256(torch.autograd.Function):
    """NHWC conv2d with forward, dgrad and wgrad all on the 256-tile MFMA kernels."""

    @staticmethod
    def forward(ctx, x, weight, bias, stride, padding, dilation):
        ctx.save_for_backward(x)
        route = getattr(x, "_pha_res_route", None)   # first conv of a routed residual block
        ctx.route = ctx.route_src = None
        if route is not None and not route.get("armed"):
            route["armed"] = True
            ctx.route = route
        elif route is not None and route.get("kind") == "conv" and not route.get("sink"):
            # the downsample shortcut's conv: hands its dx to the armed first conv's dgrad epilogue
            route["sink"] = True
            ctx.route_src = route
        ctx.weight = weight   # the parameter object itself (a leaf input): its layout cache entries match
        ctx.conf = (stride, padding, dilation, bias is not None)
        src = getattr(x, "_pha_bn_src", None)   # x is a batch norm's output: fuse its backward sums
        ctx.bn_src = src if src is not None and src[0].shape[:3] == x.shape[:3] else None
        w_okkc = _wlayout(weight, "fwd", lambda t: t.permute(0, 2, 3, 1).contiguous())
        # training: the epilogue also emits batch-norm partial statistics of y (ResNet-style
        # conv -> BN pairs then skip the BN's own statistics pass over y); PHA_CONV_BN_STATS=0 disables
        stats = _bn_stats_on() and bias is None
        return conv256_fwd(x.contiguous(), w_okkc, stride, padding, dilation, bias=bias, bn_stats=stats)

    @staticmethod
    def backward(ctx, gy):
        x, = ctx.saved_tensors
        weight = ctx.weight
        stride, padding, dilation, has_bias = ctx.conf
        gy = gy.contiguous()
        route = ctx.route
        addend = route.pop("g", None) if route is not None and route.get("sink") else None
        if route is not None:
            route["done"] = True
        dx = conv256_dgrad(gy, weight, x.shape, stride, padding, dilation,
                           bn_src=ctx.bn_src if _bn_bwd_on() else None,
                           addend=addend) if ctx.needs_input_grad[0] else None
        src = ctx.route_src
        if src is not None and dx is not None and not src.get("done"):
            src["g"] = dx   # the first conv's dgrad (still to run) adds it in its epilogue
            dx = None
        dw = conv256_wgrad(gy, x, weight.shape, stride, padding, dilation) if ctx.needs_input_grad[1] else None
        db = gy.float().sum((0, 1, 2)).to(gy.dtype) if has_bias and ctx.needs_input_grad[2] else None
        return dx, dw, db, None, None, None


def conv2d_nhwc256(x, weight, bias, stride, padding, dilation):
    return Conv2dNHWC256.apply(x, weight, bias, tuple(stride), tuple(padding), tuple(dilation))


class ConvTranspose2dNHWC256(torch.autograd.Function):
    """y = conv_transpose(x, w), w [C_in, C_out, KH, KW]: the input gradient of the convolution F
    with weight w (F maps C_out -> C_in channels) applied to x, on the 256-tile kernels (conv256_dgrad:
    stride phases stored in place); dx = F(dy) (conv256_fwd), dw = F's filter gradient with input dy
    and output gradient x (conv256_wgrad)."""

    @staticmethod
    def forward(ctx, x, weight, bias, stride, padding, dilation, out_hw):
        x = x.contiguous()
        N = x.shape[0]
        Cout = weight.shape[1]
        y = conv256_dgrad(x, weight, (N, out_hw[0], out_hw[1], Cout), stride, padding, dilation)
        if bias is not None:
            y += bias.to(y.dtype)
        ctx.save_for_backward(x)
        ctx.weight = weight
        ctx.conf = (stride, padding, dilation, bias is not None)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, = ctx.saved_tensors
        weight = ctx.weight
        stride, padding, dilation, has_bias = ctx.conf
        gy = gy.contiguous()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            w_okkc = _wlayout(weight, "fwd", lambda t: t.permute(0, 2, 3, 1).contiguous())
            dx = conv256_fwd(gy, w_okkc, stride, padding, dilation)
        if ctx.needs_input_grad[1]:
            dw = conv256_wgrad(x, gy, weight.shape, stride, padding, dilation)
        if has_bias and ctx.needs_input_grad[2]:
            db = gy.float().sum((0, 1, 2)).to(gy.dtype)
        return dx, dw, db, None, None, None, None


def conv_transpose2d_nhwc256(x, weight, bias, stride, padding, dilation, out_hw):
    return ConvTranspose2dNHWC256.apply(x, weight, bias, tuple(stride), tuple(padding), tuple(dilation), tuple(out_hw))


class LinearHip(torch.autograd.Function):
    """y = x @ W (+ b), Paddle [in, out] weight, on the 8-phase MFMA GEMM for all three products:
    forward NN (W k-outer), dX = dY W^T (NT), dW = X^T dY (both operands k-outer)."""

    @staticmethod
    def forward(ctx, x2d, w, b):
        ctx.save_for_backward(x2d, w)
        ctx.has_b = b is not None
        return gemm8p(x2d, w, a_kouter=False, b_kouter=True, bias=b)

    @staticmethod
    def backward(ctx, gy):
        x2d, w = ctx.saved_tensors
        gy = gy.contiguous()
        dx = gemm8p(gy, w, a_kouter=False, b_kouter=False) if ctx.needs_input_grad[0] else None
        dw = gemm8p(x2d, gy, a_kouter=True, b_kouter=True) if ctx.needs_input_grad[1] else None
        db = gy.float().sum(0).to(gy.dtype) if ctx.has_b and ctx.needs_input_grad[2] else None
        return dx, dw, db


def linear_ok(x, w):
    """shapes / dtypes the own-GEMM linear path takes (PHA_MATMUL_IMPL=hip)"""
    import os
    if os.environ.get("PHA_MATMUL_IMPL", "library") != "hip":
        return False
    if not (x.is_cuda and x.dtype in (torch.bfloat16, torch.float16) and w.dtype == x.dtype and w.dim() == 2):
        return False
    K, N = w.shape
    M = x.numel() // max(1, x.shape[-1])
    return (x.shape[-1] == K and M % 8 == 0 and K % 8 == 0 and N % 8 == 0 and M * K < 2 ** 32 and M * N < 2 ** 32
            and K * N < 2 ** 32 and _lib.native_available())


def linear(x, w, b=None):
    x2d = x.reshape(-1, x.shape[-1])
    if not x2d.is_contiguous():
        x2d = x2d.contiguous()
    y = LinearHip.apply(x2d, w, b)
    return y.reshape(list(x.shape[:-1]) + [w.shape[1]])


class MatmulNTHip(torch.autograd.Function):
    """y = x @ w^T with w [N, K] (tied output embedding / logits) on gemm8p: forward NT,
    dX = dY w (B k-outer), dW = dY^T X (both k-outer)."""

    @staticmethod
    def forward(ctx, x2d, w):
        ctx.save_for_backward(x2d, w)
        return gemm8p(x2d, w, a_kouter=False, b_kouter=False)

    @staticmethod
    def backward(ctx, gy):
        x2d, w = ctx.saved_tensors
        gy = gy.contiguous()
        dx = gemm8p(gy, w, a_kouter=False, b_kouter=True) if ctx.needs_input_grad[0] else None
        dw = gemm8p(gy, x2d, a_kouter=True, b_kouter=True) if ctx.needs_input_grad[1] else None
        return dx, dw


class MatmulNTPick(torch.autograd.Function):
    """y = x @ w^T (tied logits): every product on the faster of the library GEMM and the own
    kernels for its shape (ops/gemm.py mm_nt / mm_nn / mm_tn)."""

    @staticmethod
    def forward(ctx, x2d, w):
        from . import gemm as _g4
        ctx.save_for_backward(x2d, w)
        return _g4.mm_nt(x2d, w)

    @staticmethod
    def backward(ctx, gy):
        from . import gemm as _g4
        x2d, w = ctx.saved_tensors
        gy = gy.contiguous()
        dx = _g4.mm_nn(gy, w) if ctx.needs_input_grad[0] else None
        dw = _g4.mm_tn(gy, x2d) if ctx.needs_input_grad[1] else None
        return dx, dw


def matmul_nt(x, w):
    """x @ w^T: gemm8p when PHA_MATMUL_IMPL=hip admits the shapes, else per-shape own/library pick"""
    if linear_ok(x, w.t()):
        x2d = x.reshape(-1, x.shape[-1]).contiguous()
        return MatmulNTHip.apply(x2d, w).reshape(list(x.shape[:-1]) + [w.shape[0]])
    if x.is_cuda and w.dim() == 2 and x.dtype in (torch.bfloat16, torch.float16) and w.dtype == x.dtype \
            and type(x).__name__ != "DTensor" and type(w).__name__ != "DTensor":
        x2d = x.reshape(-1, x.shape[-1])
        if not x2d.is_contiguous():
            x2d = x2d.contiguous()
        return MatmulNTPick.apply(x2d, w.contiguous() if not w.is_contiguous() else w).reshape(
            list(x.shape[:-1]) + [w.shape[0]])
    return torch.matmul(x, w.t())


def matmul_kn(x, w):
    """x @ w with w [K, N] (Paddle linear weight), own GEMM when admitted, else the NT form on
    the cached transposed weight"""
    if linear_ok(x, w):
        return linear(x, w)
    if nt_forward_ok(x, w):
        return linear_nt(x, w)
    return torch.matmul(x, w)


def weight_t(w):
    """[in, out] linear weight -> cached contiguous [out, in] copy (refreshed once per optimizer
    step via the parameter version): x @ W then runs as the NT-layout GEMM, which hipBLASLt runs
    15-35 % faster than NN at the GPT shapes (tools/bench_gpt_gemms.py). The first stale copy met
    after an optimizer step refreshes EVERY stale cached copy on that device in one batched
    transpose launch, in place (pha_transpose16_batch; PHA_WT_BATCH=0: one launch per weight)."""
    if _WT_BATCH and _tr16_ok(w) and hasattr(_L(), "pha_transpose16_batch"):
        return _weight_t_batched(w)
    return _wlayout(w, "t", _transpose2d)


_WT_BATCH = __import__("os").environ.get("PHA_WT_BATCH", "1") != "0"


def _tr16_ok(t):
    return (t.dim() == 2 and t.dtype in (torch.bfloat16, torch.float16) and t.shape[0] % 8 == 0
            and t.shape[1] % 8 == 0 and t.is_contiguous() and t.is_cuda)


def _weight_t_batched(w):
    import weakref
    key = (w.data_ptr(), tuple(w.shape), w.dtype, "t")
    hit = _wlayouts.get(key)
    if hit is not None and hit[0]() is w and hit[2] == w._version:
        return hit[1]
    todo = []   # (weight, cached [out][in] buffer, key): refreshed in place
    for k, (ref, v, ver) in list(_wlayouts.items()):
        if k[3] != "t":
            continue
        wi = ref()
        if wi is None:
            _wlayouts.pop(k, None)
            continue
        if (wi._version != ver and wi.device == w.device and _tr16_ok(wi) and k[0] == wi.data_ptr()
                and tuple(v.shape) == (wi.shape[1], wi.shape[0])):
            todo.append((wi, v, k))
    if not any(k == key for _, _, k in todo):
        _wlayouts.pop(key, None)
        todo.append((w, torch.empty(w.shape[1], w.shape[0], dtype=w.dtype, device=w.device), key))
    L = _L()
    if not getattr(L, "_trb_sig", False):
        L.pha_transpose16_batch.argtypes = [c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]
        L.pha_transpose16_batch.restype = c_int
        L._trb_sig = True
    st = c_void_p(torch.cuda.current_stream(w.device).cuda_stream)
    for i in range(0, len(todo), 64):
        chunk = todo[i:i + 64]
        n = len(chunk)
        srcs = (c_void_p * n)(*[t.data_ptr() for t, _, _ in chunk])
        dsts = (c_void_p * n)(*[v.data_ptr() for _, v, _ in chunk])
        rs = (c_int * n)(*[t.shape[0] for t, _, _ in chunk])
        cs = (c_int * n)(*[t.shape[1] for t, _, _ in chunk])
        rc = L.pha_transpose16_batch(n, srcs, dsts, rs, cs, st)
        if rc != 0:
            raise RuntimeError(f"pha_transpose16_batch failed ({rc})")
    res = next(v for _, v, k in todo if k == key)
    if len(_wlayouts) + len(todo) > 4096:
        _wlayouts.clear()
        todo = [(w, res, key)]
    for t, v, k in todo:
        _wlayouts[k] = (weakref.ref(t), v, t._version)
    return res


def _transpose2d(t):
    """contiguous t^T of a 2-D 2-byte tensor on the LDS-tiled HIP transpose (torch otherwise)"""
    R, C = t.shape
    if t.dtype not in (torch.bfloat16, torch.float16) or R % 8 or C % 8 or not t.is_contiguous() or not t.is_cuda:
        return t.t().contiguous()
    out = torch.empty(C, R, dtype=t.dtype, device=t.device)
    L = _L()
    if not getattr(L, "_tr_sig", False):
        L.pha_transpose16.argtypes = [c_void_p, c_void_p, c_int, c_int, c_void_p]
        L.pha_transpose16.restype = c_int
        L._tr_sig = True
    rc = L.pha_transpose16(_ptr(t), _ptr(out), R, C, c_void_p(torch.cuda.current_stream(t.device).cuda_stream))
    if rc != 0:
        raise RuntimeError(f"pha_transpose16 failed ({rc})")
    return out


def nt_forward_ok(x, w):
    import os
    return (os.environ.get("PHA_LINEAR_NT", "1") != "0" and x.is_cuda and w.dim() == 2 and w.requires_grad
            and type(x).__name__ != "DTensor" and type(w).__name__ != "DTensor"
            and x.dtype in (torch.bfloat16, torch.float16) and w.dtype == x.dtype)


def weight_grad(x2d, gy):
    """dW = x^T @ dY for a linear layer ([in, out]) on the own persistent TN kernel (split-K
    when the [in, out] tile grid is smaller than the chip) — ops/gemm.py mm_tn"""
    from . import gemm as _g4
    return _g4.mm_tn(x2d, gy)


class LinearNT(torch.autograd.Function):
    """y = x @ W (+ b) computed as x @ (W^T)^T on the cached transposed weight (NT GEMM, bias
    in the hipBLASLt epilogue); dX = dY W^T (NT on W itself), dW = X^T dY, db by the HIP
    column-sum kernel."""

    @staticmethod
    def forward(ctx, x2d, w, b):
        ctx.save_for_backward(x2d, w)
        ctx.has_b = b is not None
        wt = weight_t(w)
        from . import gemm as _g4
        return _g4.mm_nt_bias(x2d, wt, b) if b is not None else _g4.mm_nt(x2d, wt)

    @staticmethod
    def backward(ctx, gy):
        from . import hip
        x2d, w = ctx.saved_tensors
        gy = gy.contiguous()
        from . import gemm as _g4
        dx = _g4.mm_nt(gy, w) if ctx.needs_input_grad[0] else None
        dw = db = None
        if ctx.needs_input_grad[1] and ctx.has_b and ctx.needs_input_grad[2]:
            dw, db = _g4.mm_tn_db(x2d.contiguous(), gy)   # bias gradient from the dW GEMM's B fragments
        else:
            dw = weight_grad(x2d.contiguous(), gy) if ctx.needs_input_grad[1] else None
            db = hip.col_sum(gy) if ctx.has_b and ctx.needs_input_grad[2] else None
        return dx, dw, db


def linear_nt(x, w, b=None):
    x2d = x.reshape(-1, x.shape[-1])
    return LinearNT.apply(x2d, w, b).reshape(list(x.shape[:-1]) + [w.shape[1]])
