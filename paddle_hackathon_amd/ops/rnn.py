"""The reference ``rnn`` op (paddle/fluid/operators/rnn_op.cc; phi rnn_kernel / rnn_grad_kernel):
multi-layer, optionally bidirectional SimpleRNN (tanh / relu), LSTM and GRU over a time-major
input with an optional per-row SequenceLength.

Per (layer, direction): the input projection of every time step is ONE GEMM
(``x W_ih^T + b_ih`` on the own GEMM kernels, ops/gemm.py), then the recurrence runs on the
per-step HIP kernels of csrc/kernels/rnn.hip (hidden-state product on fp32 MFMAs + the cell), and
its backward likewise; the weight gradients are GEMMs over all steps. CPU tensors take torch's
recurrent kernels (or a step loop when sequence lengths mask rows).

Weight list order is the reference's ``RNNBase._all_weights`` (rnn.py:953-962): every
(layer, direction)'s ``weight_ih, weight_hh`` first, then every ``bias_ih, bias_hh``."""
from __future__ import annotations

import ctypes

import torch

MODES = {"RNN_TANH": 0, "RNN_RELU": 1, "LSTM": 2, "GRU": 3}
GATES = {0: 1, 1: 1, 2: 4, 3: 3}


def _lib():
    from . import _lib as m
    L = m._load()
    if L is None:   # a GPU run without the kernel library fails loudly
        m.require_native()
        raise RuntimeError("paddle_hackathon_amd: HIP kernel library unavailable for the rnn op")
    if not getattr(L, "_pha_rnn_sig", False):
        p = ctypes.c_void_p
        i = ctypes.c_int
        L.pha_rnn_fwd.argtypes = [i, i, i, i, p, p, p, p, p, p, p, p, i, p]
        L.pha_rnn_fwd.restype = i
        L.pha_rnn_bwd.argtypes = [i, i, i, i, p, p, p, p, p, p, p, p, p, p, p, i, p]
        L.pha_rnn_bwd.restype = i
        L._pha_rnn_sig = True
    return L


def _p(t):
    return ctypes.c_void_p(0 if t is None else t.data_ptr())


def _stream(t):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


class _Recur(torch.autograd.Function):
    """the time loop of one (layer, direction) on the HIP kernels: gx [T, B, G*H] (x-side gate
    pre-activations, time order), h0 / c0 [B, H], w_hh [G*H, H], b_hh [G*H] -> y [T, B, H], hT, cT"""

    @staticmethod
    def forward(ctx, gx, h0, c0, w_hh, b_hh, lens, mode, reverse):
        T, B, GH = gx.shape
        H = w_hh.shape[1]
        dev = gx.device
        gx, w_hh = gx.contiguous(), w_hh.contiguous()
        hall = torch.empty(T + 1, B, H, device=dev, dtype=torch.float32)
        hall[0] = h0
        call = save = None
        if mode == 2:
            call = torch.empty(T + 1, B, H, device=dev, dtype=torch.float32)
            call[0] = c0
        if mode in (2, 3):
            save = torch.empty(T, B, 4 * H, device=dev, dtype=torch.float32)
        y = torch.empty(T, B, H, device=dev, dtype=torch.float32)
        bh = None if b_hh is None else b_hh.contiguous()
        rc = _lib().pha_rnn_fwd(mode, T, B, H, _p(gx), _p(w_hh), _p(bh), _p(lens), _p(y), _p(hall), _p(call),
                                _p(save), int(reverse), _stream(gx))
        if rc != 0:
            raise RuntimeError(f"pha_rnn_fwd failed ({rc}) mode={mode} T={T} B={B} H={H}")
        ctx.save_for_backward(w_hh, hall, call, save, lens)
        ctx.mode, ctx.reverse, ctx.has_b = mode, reverse, b_hh is not None
        hT = hall[T].clone()
        cT = call[T].clone() if mode == 2 else torch.zeros(0, device=dev)
        if mode != 2:
            ctx.mark_non_differentiable(cT)
        return y, hT, cT

    @staticmethod
    def backward(ctx, dy, dhT, dcT):
        w_hh, hall, call, save, lens = ctx.saved_tensors
        mode, reverse = ctx.mode, ctx.reverse
        T1, B, H = hall.shape
        T = T1 - 1
        GH = w_hh.shape[0]
        dev = hall.device
        dpass = dhT.float().contiguous().clone() if dhT is not None else torch.zeros(B, H, device=dev)
        dc = None
        if mode == 2:
            dc = dcT.float().contiguous().clone() if dcT is not None and dcT.numel() else torch.zeros(B, H, device=dev)
        dgx = torch.empty(T, B, GH, device=dev, dtype=torch.float32)
        dgh = torch.empty(T, B, GH, device=dev, dtype=torch.float32)
        dh0 = torch.empty(B, H, device=dev, dtype=torch.float32)
        dyc = None if dy is None else dy.float().contiguous()
        rc = _lib().pha_rnn_bwd(mode, T, B, H, _p(dyc), _p(w_hh), _p(lens), _p(hall), _p(call), _p(save), _p(dgx),
                                _p(dgh), _p(dpass), _p(dc), _p(dh0), int(reverse), _stream(hall))
        if rc != 0:
            raise RuntimeError(f"pha_rnn_bwd failed ({rc})")
        from .gemm import matmul
        dw_hh = matmul(dgh.reshape(T * B, GH), hall[:T].reshape(T * B, H), transpose_a=True)
        db_hh = dgh.sum((0, 1)) if ctx.has_b else None
        if reverse:
            dgx = dgx.flip(0)
        return dgx, dh0, dc, dw_hh, db_hh, None, None, None


def _proj(x, w_ih, b_ih):
    """x [T, B, I] -> x W_ih^T + b_ih [T, B, G*H] on the own GEMM kernels (autograd)"""
    from .gemm import matmul
    T, B, I = x.shape
    gx = matmul(x.reshape(T * B, I), w_ih, transpose_b=True)
    if b_ih is not None:
        gx = gx + b_ih
    return gx.reshape(T, B, -1)


def _recur_torch(gx, h0, c0, w_hh, b_hh, lens, mode, reverse):
    """the same recurrence as torch ops (CPU with sequence lengths; the fp32 oracle of the tests)"""
    T = gx.shape[0]
    H = w_hh.shape[1]
    h, c = h0, c0
    ys = [None] * T
    for s in range(T):
        t = T - 1 - s if reverse else s
        a = gx[t]
        hw = h @ w_hh.t() + (b_hh if b_hh is not None else 0)
        if mode == 2:
            i, f, g, o = torch.sigmoid(a[:, :H] + hw[:, :H]), torch.sigmoid(a[:, H:2 * H] + hw[:, H:2 * H]), \
                torch.tanh(a[:, 2 * H:3 * H] + hw[:, 2 * H:3 * H]), torch.sigmoid(a[:, 3 * H:] + hw[:, 3 * H:])
            cn = f * c + i * g
            hn = o * torch.tanh(cn)
        elif mode == 3:
            r = torch.sigmoid(a[:, :H] + hw[:, :H])
            z = torch.sigmoid(a[:, H:2 * H] + hw[:, H:2 * H])
            n = torch.tanh(a[:, 2 * H:] + r * hw[:, 2 * H:])
            hn, cn = z * h + (1 - z) * n, c
        else:
            hn = torch.tanh(a + hw) if mode == 0 else torch.relu(a + hw)
            cn = c
        if lens is not None:
            m = (t < lens).unsqueeze(1)
            hn = torch.where(m, hn, h)
            if mode == 2:
                cn = torch.where(m, cn, c)
            ys[t] = torch.where(m, hn, torch.zeros_like(hn))
        else:
            ys[t] = hn
        h, c = hn, cn
    return torch.stack(ys, 0), h, c


def _vf_layer(x, h0, c0, ws, mode, reverse):
    """one (layer, direction) on torch's recurrent kernel (CPU, no masking): x [T, B, I]"""
    if reverse:
        x = x.flip(0)
    has_b = len(ws) == 4
    if mode == 2:
        out, h, c = torch._VF.lstm(x, (h0.unsqueeze(0), c0.unsqueeze(0)), ws, has_b, 1, 0.0, False, False, False)
        hT, cT = h[0], c[0]
    else:
        f = torch._VF.gru if mode == 3 else (torch._VF.rnn_tanh if mode == 0 else torch._VF.rnn_relu)
        out, h = f(x, h0.unsqueeze(0), ws, has_b, 1, 0.0, False, False, False)
        hT, cT = h[0], c0
    if reverse:
        out = out.flip(0)
    return out, hT, cT


def layer(x, h0, c0, w_ih, w_hh, b_ih, b_hh, lens, mode, reverse):
    """one (layer, direction): x [T, B, I] -> (y [T, B, H], hT, cT)"""
    if x.is_cuda:
        dt = x.dtype
        gx = _proj(x.to(w_ih.dtype), w_ih, b_ih).float()
        c0f = c0.float() if mode == 2 else torch.zeros(0, device=x.device)
        y, hT, cT = _Recur.apply(gx, h0.float(), c0f, w_hh.float(), None if b_hh is None else b_hh.float(),
                                 lens, mode, bool(reverse))
        return y.to(dt), hT.to(dt), (cT.to(dt) if mode == 2 else c0)
    if lens is None:
        ws = [w_ih, w_hh] + ([b_ih, b_hh] if b_ih is not None else [])
        return _vf_layer(x, h0, c0, ws, mode, reverse)
    gx = x @ w_ih.t() + (b_ih if b_ih is not None else 0)
    return _recur_torch(gx, h0, c0, w_hh, b_hh, lens, mode, reverse)


def rnn(x, pre_state, weight_list, sequence_length, dropout_prob, is_bidirec, input_size, hidden_size, num_layers,
        mode, is_test, training_dropout=None):
    """The reference rnn op on torch tensors: x [T, B, I] time-major; pre_state [h0] or [h0, c0]
    ([L*D, B, H]); weight_list in the reference order -> (out [T, B, D*H], [h_n] or [h_n, c_n])."""
    m = MODES[mode]
    D = 2 if is_bidirec else 1
    L = num_layers
    nw = 2 * L * D
    has_b = len(weight_list) == 2 * nw
    lens = None
    if sequence_length is not None:
        lens = sequence_length.to(device=x.device, dtype=torch.int32).contiguous()
    h0 = pre_state[0]
    c0 = pre_state[1] if m == 2 else None
    hs, cs = [], []
    inp = x
    for l in range(L):
        outs = []
        for d in range(D):
            k = l * D + d
            w_ih, w_hh = weight_list[2 * k], weight_list[2 * k + 1]
            b_ih, b_hh = (weight_list[nw + 2 * k], weight_list[nw + 2 * k + 1]) if has_b else (None, None)
            y, hT, cT = layer(inp, h0[k], c0[k] if c0 is not None else torch.zeros(0, device=x.device, dtype=x.dtype),
                              w_ih, w_hh, b_ih, b_hh, lens, m, d == 1)
            outs.append(y)
            hs.append(hT)
            if m == 2:
                cs.append(cT)
        inp = outs[0] if D == 1 else torch.cat(outs, -1)
        if dropout_prob and not is_test and l < L - 1:
            inp = torch.nn.functional.dropout(inp, dropout_prob, training=True)
    state = [torch.stack(hs, 0)]
    if m == 2:
        state.append(torch.stack(cs, 0))
    return inp, state
