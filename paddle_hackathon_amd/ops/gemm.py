"""Own-GEMM entry points on the one-wave-per-SIMD 256x256x64 MFMA kernel (csrc/kernels/gemm4w.hip).

Reference behaviour: every matmul of the reference goes through
``phi/kernels/impl/matmul_kernel_impl.h:88`` (cuBLAS), the fused linear-epilogue op through
``paddle/fluid/operators/fused/fused_gemm_epilogue_op.cu:29,298`` (cuBLASLt bias/gelu/relu
forward, dgelu + bias-grad backward). Here the same products run on our own gfx950 kernel with
the epilogues folded in:

  * ``gemm(a, b, a_kouter, b_kouter, ...)``   C = op(A) @ op(B) (+bias)(gelu|relu)
      a: [M, K] (a_kouter=False) or [K, M];  b: B^T [N, K] (b_kouter=False) or B [K, N]
  * forward fc1:   h = x @ W1 + b1 stored as pre-activation AND a = gelu(h) in one pass
  * backward fc2-dgrad: dH = (dY @ W2^T) * gelu'(h) with the bias-gradient column sums of dH

Operands need K % 64 == 0 and M, N, row strides % 8 == 0 (``supported``); the ``mm_*`` entry
points zero-pad tails (K to 64, M / N to 8) so odd shapes (vocab 30522, a handful of masked
tokens, a batch of 8) stay on the own kernels.
"""
from __future__ import annotations

import os
from ctypes import c_int, c_long, c_void_p

import torch

from . import _lib

EPI_BIAS, EPI_GELU, EPI_RELU, EPI_DGELU, EPI_COLSUM, EPI_AUXOUT, EPI_TRANS = 1, 2, 4, 8, 16, 32, 64
EPI_RSTAGE = 32768   # gemm4p NT: register-staged operands
EPI_EARLY = 65536    # gemm4p: early-release schedule (read burst + buffer release early in phase A)
EPI_RING = 1 << 22   # gemm4p NT: 4-slot ring of 32-deep stages (gemm4r_kernel; K % 64 == 0, K >= 128)
EPI_ADEEP = 1 << 23  # gemm4p NT, no bias / GELU: 3 A + 2 B LDS slots (gemm4a_kernel; K >= 256)
EPI_WSTAG = 1 << 24  # gemm4p NT + EARLY: wave w issues its LDS-DMA after MFMA w of a group
G4P_COLSUM = 1 << 27  # gemm4p TN + EARLY: column sums of B (bias gradient) from the MFMA B fragments
G4P_SPREAD_SHIFT = 28  # gemm4p NT + EARLY, bits 28-29: LDS-DMA placement over 24-28 MFMA groups
_DT = {torch.bfloat16: 1, torch.float16: 2, torch.float32: 0}


def _L():
    L = _lib._load()
    if L is None:
        raise RuntimeError(f"libpha_kernels.so not loaded: {_lib._load_error}")
    if not getattr(L, "_g4w_sig", False):
        P, I, LG = c_void_p, c_int, c_long
        L.pha_gemm4w.argtypes = [I, P, P, P, LG, LG, LG, LG, LG, LG, I, I, I, P, P, LG, P, I, P]
        L.pha_gemm4w.restype = c_int
        L.pha_gemm4p.argtypes = [I, P, P, P, LG, LG, LG, LG, LG, LG, I, I, I, I, P, I, I, P, I, P, P]
        L.pha_gemm4p.restype = c_int
        L.pha_gemm4p_batched.argtypes = [I, P, P, P, LG, LG, LG, LG, LG, LG, I, I, I, I, P, I, I, P, I, P, P, I,
                                         LG, LG, LG]
        L.pha_gemm4p_batched.restype = c_int
        L.pha_gemm8w.argtypes = [I, P, P, P, LG, LG, LG, LG, LG, LG, I, P, I, P]
        L.pha_gemm8w.restype = c_int
        L.pha_colsum_finish.argtypes = [I, P, P, I, I, P]
        L.pha_colsum_finish.restype = c_int
        L._g4w_sig = True
    return L


def _ptr(t):
    return c_void_p(0 if t is None else t.data_ptr())


def _stream(t):
    return c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def sched_variant(a_kouter=False, b_kouter=False):
    """main-loop schedule: fragment reads front-loaded (0) for the both-K-outer (weight-gradient)
    layout, spread one per MFMA group (2) otherwise — the per-layout winners on MI355X
    (tools/bench_g4w.py); PHA_G4W_SCHED overrides"""
    env = os.environ.get("PHA_G4W_SCHED")
    if env is not None:
        return int(env)
    return 0 if a_kouter else 2


def supported(M, N, K, *tensors):
    """the shapes / strides the kernel takes"""
    if K % 64 or M % 8 or N % 8 or K <= 0 or M <= 0 or N <= 0:
        return False
    for t in tensors:
        if t is None:
            continue
        if not t.is_cuda or t.dtype not in (torch.bfloat16, torch.float16) or t.dim() != 2 or t.stride(1) != 1 \
                or t.stride(0) % 8:
            return False
        if t.stride(0) * 256 * 2 >= 2 ** 32 or t.data_ptr() % 16:
            return False
    return _lib.native_available()


def gemm(a, b, a_kouter=False, b_kouter=False, bias=None, act=None, aux=None, aux_out=False, colsum=False,
         out=None, trans_out=False):
    """C = epi(op(A) @ op(B)).

    trans_out (a_kouter=True, b_kouter=False only): return C^T [N, M] instead — bias is indexed
    by C^T's column (length M), colsum sums C^T's rows ([ceil(N/256), M] partials). ``nn`` below
    uses it to run x @ W as (W^T x^T)^T on the layout whose main loop keeps the accumulators in
    AGPRs.

    act: None | "gelu" | "relu" | "dgelu" (C = acc * gelu'(aux), aux = forward pre-activation).
    aux_out: with act="gelu", also write the pre-activation (acc + bias) into ``aux`` (allocated
    when None) and return it. colsum: also return the fp32 column sums of C (bias gradient).
    Returns C, or (C, aux) / (C, colsum) / (C, aux, colsum) as requested."""
    assert a.dtype in (torch.bfloat16, torch.float16) and b.dtype == a.dtype and a.dim() == 2 and b.dim() == 2
    assert a.stride(1) == 1 and b.stride(1) == 1
    M, Ka = (a.shape[1], a.shape[0]) if a_kouter else (a.shape[0], a.shape[1])
    N, Kb = (b.shape[1], b.shape[0]) if b_kouter else (b.shape[0], b.shape[1])
    assert Ka == Kb, (a.shape, b.shape, a_kouter, b_kouter)
    if trans_out:
        assert a_kouter and not b_kouter, "trans_out needs a_kouter=True, b_kouter=False"
    OM, ON = (N, M) if trans_out else (M, N)
    c = out if out is not None else torch.empty(OM, ON, dtype=a.dtype, device=a.device)
    assert c.shape == (OM, ON) and c.stride(1) == 1
    epi = 0
    if bias is not None:
        bias = bias.float().contiguous()
        epi |= EPI_BIAS
    if act == "gelu":
        epi |= EPI_GELU
    elif act == "relu":
        epi |= EPI_RELU
    elif act == "dgelu":
        assert aux is not None and aux.shape == (OM, ON) and aux.stride(1) == 1
        epi |= EPI_DGELU
    elif act is not None:
        raise ValueError(f"unknown epilogue activation {act}")
    if aux_out:
        if aux is None:
            aux = torch.empty(OM, ON, dtype=a.dtype, device=a.device)
        epi |= EPI_AUXOUT
    cs = None
    if colsum:
        cs = torch.empty((OM + 255) // 256, ON, dtype=torch.float32, device=a.device)
        epi |= EPI_COLSUM
    if trans_out:
        epi |= EPI_TRANS
    rc = _L().pha_gemm4w(_DT[a.dtype], _ptr(a), _ptr(b), _ptr(c), M, N, Ka, a.stride(0), b.stride(0), c.stride(0),
                         int(a_kouter), int(b_kouter), epi, _ptr(bias), _ptr(aux),
                         aux.stride(0) if aux is not None else 0, _ptr(cs), sched_variant(a_kouter, b_kouter), _stream(a))
    if rc != 0:
        raise RuntimeError(f"pha_gemm4w failed ({rc}) M={M} N={N} K={Ka} a_kouter={a_kouter} b_kouter={b_kouter}")
    res = [c]
    if aux_out:
        res.append(aux)
    if colsum:
        res.append(cs)
    return res[0] if len(res) == 1 else tuple(res)


def _num_cus(dev):
    return torch.cuda.get_device_properties(dev).multi_processor_count


def _group_m(a_kouter, b_kouter, K, N):
    """tile-walk panel height (M-tile rows per panel) of a gemm4p launch: 8 for NT products with
    K < 4096, measured at the bench's M = 98,304 (2048 x 2048: 667 vs 701 us at the kernel's
    default 4; 6144 x 2048: 1848 vs 1879 us; profiles/nt_mb48_r5/r5_groupm.log), else 4 (long-K NT
    is best at 4: 2289 vs 2378 us at 8; so is the 50304-wide head: 15.0 vs 16.2 ms).
    PHA_G4P_GROUP_M overrides."""
    env = os.environ.get("PHA_G4P_GROUP_M")
    if env:
        return int(env)
    return 8 if (not a_kouter and not b_kouter and K < 4096 and N <= 8192) else 4


def gemm_p(a, b, a_kouter=False, b_kouter=False, bias=None, out=None, trans_out=False, epi_extra=0, grid=0,
           group_m=0, splits=1, gelu_aux=None, colsum=False):
    """C = op(A) @ op(B) (+ bias[output column]) on the persistent epilogue-overlapped kernel
    (csrc/kernels/gemm4p.hip). Layouts: NT (False, False), TN (True, True), and with trans_out
    (True, False) the transposed product C^T [N, M] (``nn_p`` runs x @ W through it).
    splits > 1 (TN only): split-K into fp32 slabs + an in-order reduce (few-tile weight gradients).
    gelu_aux (NT only): C = gelu_tanh(A B^T + bias) and gelu_aux <- A B^T (the pre-activation
    without the bias, shaped and strided like C) from the same epilogue.
    colsum (TN only): also the column sums of B over K (a linear layer's bias gradient sum_t dY[t]),
    summed by the main loop from the B fragments it already holds; returns (C, fp32 partials
    [2 * splits * ceil(M / 256) (+ 8 workspace rows), N]) — finish with colsum_rows_finish."""
    assert a.dtype in (torch.bfloat16, torch.float16) and b.dtype == a.dtype and a.dim() == 2 and b.dim() == 2
    assert a.stride(1) == 1 and b.stride(1) == 1
    M, Ka = (a.shape[1], a.shape[0]) if a_kouter else (a.shape[0], a.shape[1])
    N, Kb = (b.shape[1], b.shape[0]) if b_kouter else (b.shape[0], b.shape[1])
    assert Ka == Kb, (a.shape, b.shape, a_kouter, b_kouter)
    assert (a_kouter, b_kouter, trans_out) in ((False, False, False), (True, True, False), (True, False, True))
    OM, ON = (N, M) if trans_out else (M, N)
    c = out if out is not None else torch.empty(OM, ON, dtype=a.dtype, device=a.device)
    assert c.shape == (OM, ON) and c.stride(1) == 1
    epi = epi_extra | _epi_default(a_kouter, b_kouter, trans_out, Ka)
    if bias is not None:
        bias = bias.float().contiguous()
        assert bias.numel() == ON
        epi |= EPI_BIAS
    ws = None
    if splits > 1:
        ws = torch.empty(splits * OM * ON, dtype=torch.float32, device=a.device)
    if gelu_aux is not None:
        assert (a_kouter, b_kouter, trans_out, splits) == (False, False, False, 1)
        assert gelu_aux.shape == c.shape and gelu_aux.stride() == c.stride() and gelu_aux.dtype == c.dtype
        epi |= EPI_GELU
    part = None
    if colsum:
        assert (a_kouter, b_kouter, trans_out) == (True, True, False) and gelu_aux is None
        # + 8 rows: the first-stage workspace of the two-stage column reduction (hip._col_sum_rows)
        part = torch.empty(2 * splits * -(-M // 256) + 8, N, dtype=torch.float32, device=a.device)
        epi |= G4P_COLSUM | EPI_EARLY
        gelu_aux = part
    if group_m <= 0:
        group_m = _group_m(a_kouter, b_kouter, Ka, N)
    rc = _L().pha_gemm4p(_DT[a.dtype], _ptr(a), _ptr(b), _ptr(c), M, N, Ka, a.stride(0), b.stride(0), c.stride(0),
                         int(a_kouter), int(b_kouter), int(trans_out), epi, _ptr(bias), grid or _num_cus(a.device),
                         group_m, _ptr(ws), splits, _stream(a), _ptr(gelu_aux))
    if rc != 0:
        raise RuntimeError(f"pha_gemm4p failed ({rc}) M={M} N={N} K={Ka} a_kouter={a_kouter} b_kouter={b_kouter}")
    return (c, part) if colsum else c


def gemm_8w(a, bt, bias=None, out=None, epi_extra=0, group_m=0):
    """C = a [M, K] @ bt [N, K]^T (+ bias) on the 8-wave (two waves per SIMD) NT kernel
    (csrc/kernels/gemm8w.hip)"""
    assert a.dtype in (torch.bfloat16, torch.float16) and bt.dtype == a.dtype and a.dim() == 2 and bt.dim() == 2
    assert a.stride(1) == 1 and bt.stride(1) == 1 and a.shape[1] == bt.shape[1]
    M, K = a.shape
    N = bt.shape[0]
    c = out if out is not None else torch.empty(M, N, dtype=a.dtype, device=a.device)
    assert c.shape == (M, N) and c.stride(1) == 1
    epi = epi_extra
    if bias is not None:
        bias = bias.float().contiguous()
        assert bias.numel() == N
        epi |= 1
    rc = _L().pha_gemm8w(_DT[a.dtype], _ptr(a), _ptr(bt), _ptr(c), M, N, K, a.stride(0), bt.stride(0), c.stride(0),
                         epi, _ptr(bias), group_m, _stream(a))
    if rc != 0:
        raise RuntimeError(f"pha_gemm8w failed ({rc}) M={M} N={N} K={K}")
    return c


def _lv_bits(lv):
    """gemm4p NT schedule variant LV -> epilogue flag bits: LV & 15 at bit 17 (late-wait / PIN /
    stamp), LV & 16 = EPI_WSTAG, (LV >> 5) & 3 at bit 28 (SPREAD DMA placement, gemm4p.hip sp_na)"""
    return ((lv & 15) << 17) | (EPI_WSTAG if lv & 16 else 0) | (((lv >> 5) & 3) << G4P_SPREAD_SHIFT)


def _epi_default(a_kouter, b_kouter, trans_out, K):
    """gemm4p main-loop schedule (bitwise-identical results either way): the early-release schedule
    on every layout — phase A's fragment reads in a burst over 8 MFMA groups, the LDS buffer
    released there, the next-next K-tile's DMAs spread over the following 16 groups. 8-9 % faster on
    long-K NT, ~1 % on the TN weight gradients and K = 2048 NT, +0.3-0.4 % on the whole GPT step
    (profiles/gemm4p_early_ab_r3.log, gemm4p_relg_ab_r3.log). PHA_G4P_EARLY=0 selects the plain
    schedule (1 forces the early one)."""
    if os.environ.get("PHA_G4P_EARLY", "1") == "0":
        return 0
    if not (a_kouter or b_kouter or trans_out):
        # NT: PIN variant (LV 8 — an empty memory asm closes every MFMA group so no IR pass sinks
        # a group's LDS reads past the loop latch): 1-3 % over LV 0 on every GPT NT shape in bursts,
        # bitwise identical (profiles/g4p_late_ab_r5.log), plus SPREAD (LV 40: the next-next K-tile's
        # DMAs over 24 MFMA groups instead of 16): 1-3 % on long K, level at K = 2048, +0.2 % on the
        # library-free GPT step (profiles/g4p_spread_r6/); PHA_G4P_LV overrides. Long-K products
        # without an epilogue take the A-deep build (3 A + 2 B LDS slots, ~2 K-tiles of cover for the
        # streamed activation panel): 2.5-3 % faster at K >= 6144 under sustained load, bitwise
        # equal (profiles/g4p_adeep_sustain_r5.log); the kernel picks it only without bias / GELU
        lv = _lv_bits(int(os.environ.get("PHA_G4P_LV", "40")))
        if K >= 4096 and os.environ.get("PHA_G4P_ADEEP", "1") != "0":
            return EPI_EARLY | lv | EPI_ADEEP
        return EPI_EARLY | lv
    if a_kouter and b_kouter:
        # TN (weight gradients, unsplit): PIN + SPREAD (LV 40) — GPT-3 1.3B qkv / fc1 / fc2 dW 4.3 / 1.2 /
        # 1.8 % faster than the plain early schedule, bitwise equal (profiles/tn_lv_r6/tn_lv_ab.log)
        return EPI_EARLY | _lv_bits(int(os.environ.get("PHA_G4P_TN_LV", "40")))
    return EPI_EARLY


def nn_p(a, b, bias=None, **kw):
    """a [M, K] @ b [K, N] (+ bias) on the persistent kernel as (b^T a^T)^T"""
    return gemm_p(b, a, True, False, bias=bias, trans_out=True, **kw)


def colsum_rows_finish(part, dtype):
    """column sums of gemm_p(colsum=True)'s partials (all rows but the last 8, the workspace) on the
    two-stage HIP column reduction: row blocks in parallel, then one pass over their sums (the
    one-thread-per-column colsum_finish walked up to 2 x 16 x tiles rows serially on 3-12
    workgroups: 2.2 ms per BERT step)"""
    from . import hip as _hip
    return _hip._col_sum_rows(part, part.shape[0] - 8, dtype)


def colsum_finish(part, dtype):
    """[rows, N] fp32 partial column sums -> [N] in ``dtype``"""
    rows, N = part.shape
    out = torch.empty(N, dtype=dtype, device=part.device)
    rc = _L().pha_colsum_finish(_DT[dtype], _ptr(part), _ptr(out), rows, N, _stream(part))
    if rc != 0:
        raise RuntimeError(f"pha_colsum_finish failed ({rc})")
    return out


# ----------------------------------------------------------------------------------------------
# kernel selection: static and deterministic (same choice on every rank and every run)
# ----------------------------------------------------------------------------------------------
# PHA_GEMM_IMPL selects per layout, statically (profiles/gemm_paths_r3.log, per GPT-1.3B shape):
#   "auto" (default) — weight gradients (TN, split-K when the tile grid is smaller than the chip)
#       and NN products on the own gemm4p kernel, where it beats hipBLASLt by 4-16 %; the NT
#       forward / dX products on hipBLASLt, which is 3-21 % faster there (long-K NT is latency
#       bound on gemm4p's two-stage LDS ring);
#   "own" — every supported product on gemm4p (what the zero-library traces use);
#   "library" — every product on hipBLASLt.
# Shapes the own kernel cannot take always go to the library and are counted by ops/fallback.py.
def _impl():
    return os.environ.get("PHA_GEMM_IMPL", "auto")


_AUTO_OWN = ("tn", "nn")


def bmm_p(a, b, a_kouter=False, b_kouter=False, trans_out=False):
    """batched C_i = op(A_i) @ op(B_i) on ONE persistent gemm4p launch (the tiles of every item share
    the grid): a / b are [batch, ., .] with unit inner stride, layouts as ``gemm_p``. Batch strides
    may be 0 (a broadcast operand)."""
    assert a.dim() == 3 and b.dim() == 3 and a.shape[0] == b.shape[0]
    assert a.stride(2) == 1 and b.stride(2) == 1
    Bn = a.shape[0]
    M, Ka = (a.shape[2], a.shape[1]) if a_kouter else (a.shape[1], a.shape[2])
    N, Kb = (b.shape[2], b.shape[1]) if b_kouter else (b.shape[1], b.shape[2])
    assert Ka == Kb
    assert (a_kouter, b_kouter, trans_out) in ((False, False, False), (True, True, False), (True, False, True))
    OM, ON = (N, M) if trans_out else (M, N)
    c = torch.empty(Bn, OM, ON, dtype=a.dtype, device=a.device)
    epi = _epi_default(a_kouter, b_kouter, trans_out, Ka)
    rc = _L().pha_gemm4p_batched(_DT[a.dtype], _ptr(a), _ptr(b), _ptr(c), M, N, Ka, a.stride(1), b.stride(1),
                                 c.stride(1), int(a_kouter), int(b_kouter), int(trans_out), epi, None,
                                 _num_cus(a.device), 0, None, 1, _stream(a), None, Bn, a.stride(0), b.stride(0),
                                 c.stride(0))
    if rc != 0:
        raise RuntimeError(f"pha_gemm4p_batched failed ({rc}) batch={Bn} M={M} N={N} K={Ka}")
    return c


def _bmm_ok(t):
    """a [batch, R, C] view the batched kernel reads directly: unit stride on one of the two inner
    dims, 16-B aligned rows and batch offsets, 32-bit tile offsets"""
    if not (t.is_cuda and t.dtype in (torch.bfloat16, torch.float16) and t.dim() == 3 and t.data_ptr() % 16 == 0):
        return False
    s0, s1, s2 = t.stride()
    ld = s1 if s2 == 1 else (s2 if s1 == 1 else -1)
    return ld > 0 and ld % 8 == 0 and s0 % 8 == 0 and s0 >= 0 and ld * 256 * 2 < 2 ** 32


def bmm_own(a, b):
    """C [batch, M, N] = a [batch, M, K] @ b [batch, K, N] on the batched own kernel, each operand
    row-major or transposed (column-major) in its last two dims; None when the operands do not fit
    (K % 64, M / N % 8, strides)"""
    Bn, M, K = a.shape
    N = b.shape[2]
    if K % 64 or M % 8 or N % 8 or not (_bmm_ok(a) and _bmm_ok(b)) or not _lib.native_available():
        return None
    a_row, b_row = a.stride(2) == 1, b.stride(2) == 1
    if a_row and b_row:        # NN: C^T = B^T A^T through the transposed store
        return bmm_p(b, a, True, False, trans_out=True)
    if a_row:                  # b^T [N, K] row-major: NT
        return bmm_p(a, b.transpose(1, 2), False, False)
    if b_row:                  # a^T [K, M] row-major: TN
        return bmm_p(a.transpose(1, 2), b, True, True)
    # both transposed: C^T = B^T A^T as NN on the row-major views
    return bmm_p(a.transpose(1, 2), b.transpose(1, 2), True, False, trans_out=True).transpose(1, 2)


class _BMM(torch.autograd.Function):
    """C = A @ B per batch item; dA = dC B^T, dB = A^T dC (transposed views, no copies)"""

    @staticmethod
    def forward(ctx, a, b):
        ctx.save_for_backward(a, b)
        return bmm_own(a, b)

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        g = g if g.stride(2) == 1 or g.stride(1) == 1 else g.contiguous()
        da = db = None
        if ctx.needs_input_grad[0]:
            da = bmm_own(g, b.transpose(1, 2))
            if da is None:
                da = torch.bmm(g, b.transpose(1, 2))
        if ctx.needs_input_grad[1]:
            db = bmm_own(a.transpose(1, 2), g)
            if db is None:
                db = torch.bmm(a.transpose(1, 2), g)
        return da, db


def _bmm_fits(x3, y3):
    return (x3.dim() == 3 and y3.dim() == 3 and x3.shape[2] % 64 == 0 and x3.shape[1] % 8 == 0
            and y3.shape[2] % 8 == 0 and _bmm_ok(x3) and _bmm_ok(y3))


# NT shapes (N, K) where gemm4p matches hipBLASLt in isolation at the bench's M = 98,304: the GPT-3
# 1.3B qkv forward, 1830 vs 1842 us (profiles/nt_mb48_r5/r5_nt_mb48_gm8.log). Opt-in
# (PHA_GEMM_AUTO_NT_OWN=1): inside the training step it measured -0.55 % (125.5k vs 126.2k
# tokens/s, three alternating pairs, profiles/nt_mb48_r5/)
_AUTO_OWN_NT_SHAPES = {(6144, 2048)}


def _auto_own_nt(N, K):
    """NT products the auto policy puts on gemm4p, both opt-in: the isolated ties above
    (PHA_GEMM_AUTO_NT_OWN=1), and (PHA_GEMM_AUTO_NT=1) N <= 2048 and K <= 2048 (the attention output projection's forward and
    dX, 204 vs 206 us at 32768x2048x2048, profiles/gemm4p_early_ab_r3.log, but 10 % behind at
    M = 98,304); the other NT products stay on the library, 3-10 % faster"""
    if (N, K) in _AUTO_OWN_NT_SHAPES and os.environ.get("PHA_GEMM_AUTO_NT_OWN", "0") == "1":
        return True
    return N <= 2048 and K <= 2048 and os.environ.get("PHA_GEMM_AUTO_NT", "0") == "1"


def _own_ok(layout, *ts, shape=None):
    impl = _impl()
    if impl == "auto" and layout == "nt" and shape is not None and _auto_own_nt(*shape):
        impl = "own"
    if impl == "library" or (impl == "auto" and layout not in _AUTO_OWN):
        return False
    return all(t.is_cuda and t.dtype in (torch.bfloat16, torch.float16) and t.dim() == 2 for t in ts) \
        and _lib.native_available()


def _c(t):
    return t if t.stride(1) == 1 else t.contiguous()


def _lib_call(layout, name, shape, fn):
    """every product that leaves the own kernels is counted: as a fallback when the policy wanted
    the own kernel (unsupported operands), as a planned library product otherwise (``auto`` NT,
    ``library``) — ops/fallback.py keeps the two apart"""
    from . import fallback
    impl = _impl()
    if impl == "own" or (impl == "auto" and layout in _AUTO_OWN):
        fallback.note("matmul", f"{name} {shape} unsupported by the own kernels -> library")
    else:
        fallback.library("matmul", f"{name} {shape} on hipBLASLt (PHA_GEMM_IMPL={impl})")
    return fn()


def _splits(M, N, K, dev):
    """split-K factor for a weight gradient: grids of >= 2 rounds stay unsplit, and so do grids of
    >= 3/4 of a round (the qkv dW's 192 tiles unsplit beat split 4: 714 vs 739 us sustained,
    profiles/tn_wgrad_r5/tn_sustain.log). Below that, the power of two (<= 16, dividing the K-tiles,
    >= 4 K-tiles per item) with the least modelled time: rounds of work items x K-tiles per item x
    0.76 us (one K-tile of a 256 x 256 tile) + splits x tiles x 0.12 us (each item's fp32 slab written
    and read back by the in-order reduce). Filling every CU is not the goal: BERT-base's fc1 / fc2
    dW (36 tiles, 256 K-tiles) run 116 us at split 4 (144 items on 256 CUs) vs 164 us at the old
    fill-the-rounds pick of 16, qkv dW 89.5 (split 8) vs 122 us (profiles/bert_tn_ab_r6.log)."""
    tiles = -(-M // 256) * -(-N // 256)
    cus = _num_cus(dev)
    ktiles = K // 64
    if tiles >= 2 * cus or 4 * tiles >= 3 * cus:
        return 1
    best, best_t = 1, None
    sp = 1
    while sp <= 16 and ktiles % sp == 0 and ktiles // sp >= 4:
        t = -(-tiles * sp // cus) * (ktiles // sp) * 0.76 + (sp > 1) * sp * tiles * 0.12
        if best_t is None or t < best_t:
            best, best_t = sp, t
        sp *= 2
    return best


def _pad2(t, rm, cm):
    """zero-padded contiguous copy of 2-D ``t`` with rows % rm == 0 and cols % cm == 0 (t itself
    when already aligned): K tails must read zeros, and M / N / row strides need 16-B alignment"""
    R, C = t.shape
    Rp, Cp = -(-R // rm) * rm, -(-C // cm) * cm
    if (Rp, Cp) == (R, C) and t.stride(0) % 8 == 0 and t.data_ptr() % 16 == 0:
        return t
    out = torch.zeros(Rp, Cp, dtype=t.dtype, device=t.device)
    out[:R, :C] = t
    return out


def _own_fits(t):
    """the padded row stride still fits the kernel's 32-bit tile offsets"""
    return (t.shape[1] + 64) * 256 * 2 < 2 ** 32


def mm_nt(a, bt):
    """a [M, K] @ bt[N, K]^T"""
    M, K = a.shape
    N = bt.shape[0]
    if _own_ok("nt", a, bt, shape=(N, K)) and bt.dtype == a.dtype:
        a, bt = _c(a), _c(bt)
        if supported(M, N, K, a, bt):
            return gemm_p(a, bt, False, False)
        if _own_fits(a) and _own_fits(bt):
            return gemm_p(_pad2(a, 8, 64), _pad2(bt, 8, 64), False, False)[:M, :N]
    return _lib_call("nt", "nt", (M, N, K), lambda: a @ bt.t())


def mm_nt_bias(a, bt, bias):
    """a [M, K] @ bt[N, K]^T + bias (bias folded into the own kernel's epilogue)"""
    M, K = a.shape
    N = bt.shape[0]
    if _own_ok("nt", a, bt, shape=(N, K)) and bt.dtype == a.dtype:
        a, bt = _c(a), _c(bt)
        if supported(M, N, K, a, bt):
            return gemm_p(a, bt, False, False, bias=bias)
        if _own_fits(a) and _own_fits(bt):
            bp = bias if N % 8 == 0 else torch.nn.functional.pad(bias.float(), (0, -(-N // 8) * 8 - N))
            return gemm_p(_pad2(a, 8, 64), _pad2(bt, 8, 64), False, False, bias=bp)[:M, :N]
    return _lib_call("nt", "nt+bias", (M, N, K), lambda: torch.addmm(bias, a, bt.t()))


def nn(a, b, **epi):
    """a [M, K] @ b [K, N] (+ epilogue) on gemm4w as (b^T a^T)^T: A = b (K-outer), B^T = a,
    transposed store (the fused GELU / dGELU epilogue builds)"""
    return gemm(b, a, True, False, trans_out=True, **epi)


def mm_nt_bias_gelu(a, bt, bias):
    """(gelu_tanh(a bt^T + bias), a bt^T) in one own-kernel pass (the MLP's fc1 forward), or None
    when the own kernel does not take the operands"""
    M, K = a.shape
    N = bt.shape[0]
    if not (_impl() != "library" and a.is_cuda and bt.dtype == a.dtype and a.dtype in (torch.bfloat16, torch.float16)
            and supported(M, N, K, a, bt) and bias is not None and bias.numel() == N):
        return None
    pre = torch.empty(M, N, dtype=a.dtype, device=a.device)
    act = gemm_p(a, bt, False, False, bias=bias, gelu_aux=pre)
    return act, pre


def mm_nn(a, b):
    """a [M, K] @ b [K, N]"""
    M, K = a.shape
    N = b.shape[1]
    if _own_ok("nn", a, b) and b.dtype == a.dtype:
        a, b = _c(a), _c(b)
        if supported(M, N, K, a, b):
            return nn_p(a, b)
        if _own_fits(a) and _own_fits(b):
            return nn_p(_pad2(a, 8, 64), _pad2(b, 64, 8))[:M, :N]
    return _lib_call("nn", "nn", (M, N, K), lambda: a @ b)


def mm_tn(a, b):
    """a [K, M]^T @ b [K, N] (weight gradients: x^T dY), split-K when the tile grid is small"""
    K, M = a.shape
    N = b.shape[1]
    if _own_ok("tn", a, b) and b.dtype == a.dtype:
        a, b = _c(a), _c(b)
        if supported(M, N, K, a, b):
            return gemm_p(a, b, True, True, splits=_splits(M, N, K, a.device))
        if _own_fits(a) and _own_fits(b):
            ap, bp = _pad2(a, 64, 8), _pad2(b, 64, 8)
            return gemm_p(ap, bp, True, True, splits=_splits(ap.shape[1], bp.shape[1], ap.shape[0], a.device))[:M, :N]
    return _lib_call("tn", "tn", (M, N, K), lambda: a.t() @ b)


def mm_tn_db(a, b, db_dtype=None):
    """(a [K, M]^T @ b [K, N], column sums of b over K) — a linear layer's weight and bias gradients
    (x^T dY, sum_t dY[t]) from ONE pass over dY: the persistent TN kernel sums the B fragments it
    feeds to the MFMAs (v_dot2 against 1.0, each tile row of the grid taking 1/tiles_m of the K
    range) instead of a separate column-sum kernel re-reading dY from HBM.
    Reference: fused_gemm_epilogue_op.cu:298 (the bias gradient of the fused linear backward)."""
    K, M = a.shape
    N = b.shape[1]
    if _own_ok("tn", a, b) and b.dtype == a.dtype and os.environ.get("PHA_TN_COLSUM", "1") != "0":
        a, b = _c(a), _c(b)
        if supported(M, N, K, a, b):
            c, part = gemm_p(a, b, True, True, splits=_splits(M, N, K, a.device), colsum=True)
            return c, colsum_rows_finish(part, db_dtype or b.dtype)
    from . import hip as _hip
    return mm_tn(a, b), _hip.col_sum(b, db_dtype)


# ----------------------------------------------------------------------------------------------
# generic products (paddle.matmul / mm / bmm, bias-less F.linear): every bf16 / fp16 GPU product
# goes through the layouts above (own kernels under PHA_GEMM_IMPL=own, the static per-layout
# policy under auto); what cannot (fp32, batched with per-batch right operands, both operands
# transposed) is counted by ops/fallback.py. Reference: phi/kernels/impl/matmul_kernel_impl.h:88
# (MatMulFunction: 2-D, broadcast-batched and transposed forms) and :489 (MatmulGradKernel).
# ----------------------------------------------------------------------------------------------
class _NN(torch.autograd.Function):
    """C = A [M, K] @ B [K, N]; dA = dC B^T (NT on B), dB = A^T dC (TN)"""

    @staticmethod
    def forward(ctx, a, b):
        ctx.save_for_backward(a, b)
        return mm_nn(a, b)

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        g = _c(g)
        return (mm_nt(g, b) if ctx.needs_input_grad[0] else None,
                mm_tn(a, g) if ctx.needs_input_grad[1] else None)


class _NT(torch.autograd.Function):
    """C = A [M, K] @ Bt [N, K]^T; dA = dC Bt (NN), dBt = dC^T A (TN)"""

    @staticmethod
    def forward(ctx, a, bt):
        ctx.save_for_backward(a, bt)
        return mm_nt(a, bt)

    @staticmethod
    def backward(ctx, g):
        a, bt = ctx.saved_tensors
        g = _c(g)
        return (mm_nn(g, bt) if ctx.needs_input_grad[0] else None,
                mm_tn(g, a) if ctx.needs_input_grad[1] else None)


class _TN(torch.autograd.Function):
    """C = At [K, M]^T @ B [K, N]; dAt = B dC^T (NT), dB = At dC (NN)"""

    @staticmethod
    def forward(ctx, at, b):
        ctx.save_for_backward(at, b)
        return mm_tn(at, b)

    @staticmethod
    def backward(ctx, g):
        at, b = ctx.saved_tensors
        g = _c(g)
        return (mm_nt(b, g) if ctx.needs_input_grad[0] else None,
                mm_nn(at, g) if ctx.needs_input_grad[1] else None)


class _F32MM(torch.autograd.Function):
    """fp32 C = A [M, K] @ B [K, N] on the bf16 MFMA kernels: A = Ah + Al, B = Bh + Bl and
    A B ~= Ah Bh + Ah Bl + Al Bh as ONE K-outer product over 3K ([Ah; Ah; Al]^T [Bh; Bl; Bh]) with
    fp32 split-K partials (gemm256_tn); dA = dC B^T and dB = A^T dC the same way. The dropped
    Al Bl term is ~2^-16 of each product: near-fp32 results at the bf16 matrix rate."""

    @staticmethod
    def forward(ctx, a, b):
        ctx.save_for_backward(a, b)
        return mm_f32(a, b)

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        g = g.float()
        return (mm_f32(g, b.t()) if ctx.needs_input_grad[0] else None,
                mm_f32(a.t(), g) if ctx.needs_input_grad[1] else None)


def mm_f32(a, b):
    """fp32 a [M, K] @ b [K, N] (any strides) as a three-term bf16 product, fp32 out"""
    from .conv_gemm import split3, gemm256_tn
    M, K = a.shape
    N = b.shape[1]
    at3 = split3(a.t().contiguous(), 0, "hhl")        # [3K, M] (one transpose copy, then one split pass)
    b3 = split3(b.contiguous(), 0, "hlh")             # [3K, N]
    pm, pn = -M % 8, -N % 8
    if pm:
        at3 = torch.nn.functional.pad(at3, [0, pm])
    if pn:
        b3 = torch.nn.functional.pad(b3, [0, pn])
    out = gemm256_tn(at3.contiguous(), b3.contiguous(), out_dtype=torch.float32)
    return out[:M, :N] if (pm or pn) else out


def _f32_ok(a, b):
    return (a.is_cuda and b.is_cuda and a.dtype == torch.float32 and b.dtype == torch.float32
            and os.environ.get("PHA_MATMUL_F32", "hip") == "hip" and _lib.native_available())


def _gemm_dtype_ok(a, b):
    return (a.is_cuda and b.is_cuda and a.dtype in (torch.bfloat16, torch.float16) and b.dtype == a.dtype
            and type(a).__name__ != "DTensor" and type(b).__name__ != "DTensor" and _lib.native_available())


def matmul(a, b, transpose_a=False, transpose_b=False):
    """torch.matmul semantics (vectors, broadcast batches, optional transposes of the last two dims);
    2-D products — and batched left operands against a shared 2-D right operand, flattened into M —
    run on the own GEMM layouts"""
    if not (a.is_cuda or b.is_cuda):
        x = a.transpose(-1, -2) if transpose_a and a.dim() > 1 else a
        y = b.transpose(-1, -2) if transpose_b and b.dim() > 1 else b
        return torch.matmul(x, y)
    if _gemm_dtype_ok(a, b) and a.dim() >= 2 and b.dim() == 2 and not (transpose_a and transpose_b) \
            and (a.dim() == 2 or not transpose_a):
        if transpose_a:                       # a [K, M]
            return _TN.apply(_c(a), _c(b)) if not transpose_b else None
        lead = a.shape[:-1]
        a2 = _c(a.reshape(-1, a.shape[-1]))
        out = _NT.apply(a2, _c(b)) if transpose_b else _NN.apply(a2, _c(b))
        return out.reshape(*lead, out.shape[-1])
    if _gemm_dtype_ok(a, b) and a.dim() >= 3 and b.dim() >= 3 and _impl() != "library":
        # batched right operands: one persistent launch over every item's tiles (broadcast batch
        # dims as stride-0 views, no copies)
        x = a.transpose(-1, -2) if transpose_a else a
        y = b.transpose(-1, -2) if transpose_b else b
        lead = torch.broadcast_shapes(x.shape[:-2], y.shape[:-2])
        xe, ye = x.expand(*lead, *x.shape[-2:]), y.expand(*lead, *y.shape[-2:])
        x3 = xe.reshape(-1, *x.shape[-2:]) if xe.dim() != 3 else xe
        y3 = ye.reshape(-1, *y.shape[-2:]) if ye.dim() != 3 else ye
        if _bmm_fits(x3, y3):
            out = _BMM.apply(x3, y3)
            return out.reshape(*lead, *out.shape[-2:])
    if _f32_ok(a, b) and a.dim() >= 2 and b.dim() == 2 and (a.dim() == 2 or not transpose_a):
        x = a.transpose(-1, -2) if transpose_a else a
        y = b.transpose(-1, -2) if transpose_b else b
        lead = x.shape[:-1]
        out = _F32MM.apply(x.reshape(-1, x.shape[-1]), y)
        return out.reshape(*lead, out.shape[-1])
    from . import fallback
    why = (f"{a.dtype} product" if not _gemm_dtype_ok(a, b) else
           f"batched product {tuple(a.shape)} x {tuple(b.shape)}")
    fallback.note("matmul", why + " on the library")
    x = a.transpose(-1, -2) if transpose_a and a.dim() > 1 else a
    y = b.transpose(-1, -2) if transpose_b and b.dim() > 1 else b
    return torch.matmul(x, y)
