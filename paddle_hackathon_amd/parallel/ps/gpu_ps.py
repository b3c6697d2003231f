"""GPU parameter server: sparse embedding tables resident in HBM, sharded over the GPUs of the job.

Reference: paddle/fluid/framework/fleet/heter_ps/ (HeterComm: per-GPU hash tables, keys routed to
their owner GPU, pull/push over NVLink; hashtable_kernel.cu; optimizer.cuh.h sparse AdaGrad) and
python/paddle/distributed/ps (the `ps_gpu` / HeterPS training mode).

MI355X design: 288 GB of HBM3E per GPU holds the hot sparse table on the GPUs themselves. Each
rank owns the keys with ``key % world == rank`` in an open-addressing hash table in its HBM
(``csrc/kernels/gpu_ps.hip``: 64-bit CAS inserts, rows initialised from a hash of the key, fused
AdaGrad push). A pull de-duplicates the batch's ids, routes them to their owners with ONE
all-to-all (RCCL over xGMI), the owners find-or-insert and gather the rows, and a second
all-to-all returns them; a push sums duplicate gradients locally and routes them the same way.
On a CPU-only process (gloo tests) the same protocol runs over a host dict with bit-identical
initial values and update rule, so the exchange logic is testable without a GPU; on a GPU the
HIP kernels are the only path (``native_required``)."""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as tdist

from ...framework.core import Tensor, _wrap

__all__ = ["GpuPsTable", "GpuPsEmbedding"]

_EMPTY = -1     # int64 bit pattern of the kernel's ~0 key
_TOMB = -2      # ~0 - 1: a slot whose insert overflowed the row budget


def _mix64_np(x):
    x = x.astype(np.uint64)
    with np.errstate(over="ignore"):
        x = x ^ (x >> np.uint64(30))
        x = x * np.uint64(0xbf58476d1ce4e5b9)
        x = x ^ (x >> np.uint64(27))
        x = x * np.uint64(0x94d049bb133111eb)
        return x ^ (x >> np.uint64(31))


def _init_rows_np(keys, dim, seed, init_range):
    """the kernel's init_val for a batch of keys -> [n, dim] float32"""
    k = keys.astype(np.int64).view(np.uint64)[:, None]
    j = (np.arange(dim, dtype=np.uint64) + np.uint64(1))[None, :]
    with np.errstate(over="ignore"):
        h = _mix64_np(k ^ (np.uint64(seed) << np.uint64(32)) ^ (j * np.uint64(0x9e3779b97f4a7c15)))
    u = (h >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / 16777216.0)
    return ((2.0 * u - 1.0) * init_range).astype(np.float32)


class GpuPsTable:
    def __init__(self, dim, max_rows, capacity=None, lr=0.05, initial_g2sum=3.0, initial_range=1e-4,
                 bounds=(-10.0, 10.0), seed=0, device=None, group=None):
        self.dim, self.max_rows = int(dim), int(max_rows)
        cap = 1
        while cap < 2 * self.max_rows:
            cap *= 2
        self.capacity = int(capacity or cap)
        if self.capacity & (self.capacity - 1):
            raise ValueError("capacity must be a power of two")
        self.lr, self.ig2, self.init_range, self.seed = float(lr), float(initial_g2sum), float(initial_range), int(seed)
        self.lo, self.hi = bounds
        self.group = group
        self.world = tdist.get_world_size(group) if tdist.is_initialized() else 1
        self.rank = tdist.get_rank(group) if tdist.is_initialized() else 0
        from ...framework import core
        self.device = torch.device(device) if device is not None else core.default_device()
        self.gpu = self.device.type == "cuda"
        if self.gpu:
            from ...ops import _lib
            if not _lib.native_available():
                raise RuntimeError("GpuPsTable on a GPU needs the HIP kernel library (libpha_kernels.so)")
            self.keys = torch.full((self.capacity,), _EMPTY, dtype=torch.int64, device=self.device)
            self.rows = torch.full((self.capacity,), -1, dtype=torch.int32, device=self.device)
            self.next_row = torch.zeros(1, dtype=torch.int32, device=self.device)
        else:
            self._map = {}
        self.W = torch.zeros(self.max_rows, self.dim, dtype=torch.float32, device=self.device)
        self.g2 = torch.zeros(self.max_rows, dtype=torch.float32, device=self.device)

    # ------------------------------------------------------------------ local (owner) side
    def _find(self, keys, create):
        """unique int64 keys owned here -> row indices (int32; -1 absent)"""
        n = keys.numel()
        if n == 0:
            return torch.zeros(0, dtype=torch.int32, device=self.device)
        if self.gpu:
            from ...ops.hip import _L, _ptr, _stream
            from ctypes import c_float, c_int, c_long, c_uint, c_void_p
            L = _L()
            if not getattr(L, "_gps_sig", False):
                L.pha_ps_gpu_find.argtypes = [c_void_p, c_void_p, c_long, c_void_p, c_void_p, c_long, c_void_p, c_int,
                                              c_int, c_void_p, c_void_p, c_int, c_uint, c_float, c_void_p]
                L.pha_ps_gpu_find.restype = c_int
                L.pha_ps_gpu_adagrad.argtypes = [c_void_p, c_void_p, c_long, c_void_p, c_void_p, c_int, c_float,
                                                 c_float, c_float, c_float, c_void_p]
                L.pha_ps_gpu_adagrad.restype = c_int
                L._gps_sig = True
            keys = keys.contiguous()
            if bool(((keys == _EMPTY) | (keys == _TOMB)).any()):
                raise ValueError("GPU-PS keys -1 and -2 are reserved (empty / tombstone slot markers)")
            rows = torch.empty(n, dtype=torch.int32, device=self.device)
            rc = L.pha_ps_gpu_find(_ptr(keys), _ptr(rows), n, _ptr(self.keys), _ptr(self.rows), self.capacity,
                                   _ptr(self.next_row), self.max_rows, int(create), _ptr(self.W), _ptr(self.g2),
                                   self.dim, self.seed, self.init_range, _stream(self.W))
            if rc != 0:
                raise RuntimeError(f"pha_ps_gpu_find failed ({rc})")
            if create and bool((rows < -1).any()):
                raise MemoryError(f"GPU-PS table full ({self.max_rows} rows / capacity {self.capacity})")
            return rows
        ks = keys.tolist()
        out = np.empty(n, np.int32)
        new = []
        for i, k in enumerate(ks):
            r = self._map.get(k)
            if r is None and create:
                r = len(self._map)
                if r >= self.max_rows:
                    raise MemoryError(f"GPU-PS table full ({self.max_rows} rows)")
                self._map[k] = r
                new.append((i, r))
            out[i] = -1 if r is None else r
        if new:
            idx = np.array([i for i, _ in new])
            rr = torch.as_tensor(np.array([r for _, r in new]), dtype=torch.long)
            self.W[rr] = torch.from_numpy(_init_rows_np(np.asarray(ks, np.int64)[idx], self.dim, self.seed,
                                                        self.init_range))
            self.g2[rr] = 0.0
        return torch.from_numpy(out)

    def _gather(self, keys, create):
        # keys routed from several ranks may repeat: the hash kernel must see each key once per call
        uk, inv = torch.unique(keys, return_inverse=True)
        rows = self._find(uk, create).long()[inv]
        vals = self.W.index_select(0, rows.clamp_min(0))
        if not create:
            vals[rows < 0] = 0.0
        return vals

    def _update(self, keys, grads):
        # the same key may arrive from several ranks: one update with the summed gradient
        keys, inv = torch.unique(keys, return_inverse=True)
        grads = torch.zeros(keys.numel(), self.dim, dtype=torch.float32, device=self.device).index_add_(
            0, inv, grads.float())
        rows = self._find(keys, False)
        if self.gpu:
            from ...ops.hip import _L, _ptr, _stream
            g = grads.float().contiguous()
            rc = _L().pha_ps_gpu_adagrad(_ptr(rows), _ptr(g), rows.numel(), _ptr(self.W), _ptr(self.g2), self.dim,
                                         self.lr, self.ig2, float(self.lo), float(self.hi), _stream(self.W))
            if rc != 0:
                raise RuntimeError(f"pha_ps_gpu_adagrad failed ({rc})")
            return
        ok = rows >= 0
        r = rows[ok].long()
        g = grads[ok].float()
        ratio = self.lr * torch.sqrt(self.ig2 / (self.ig2 + self.g2[r]))
        self.W[r] = (self.W[r] - ratio[:, None] * g).clamp(self.lo, self.hi)
        self.g2[r] += (g * g).mean(1)

    # ------------------------------------------------------------------ routing (all-to-all)
    def _route(self, uniq):
        """-> (keys this rank must serve, per-source counts, permutation of uniq into owner order,
        send counts)"""
        owner = torch.remainder(uniq, self.world)
        order = torch.argsort(owner, stable=True)
        send = torch.bincount(owner, minlength=self.world)
        recv = torch.empty_like(send)
        tdist.all_to_all_single(recv, send, group=self.group)
        keys_in = torch.empty(int(recv.sum()), dtype=torch.int64, device=uniq.device)
        tdist.all_to_all_single(keys_in, uniq[order].contiguous(), recv.tolist(), send.tolist(), group=self.group)
        return keys_in, recv, order, send

    def pull(self, ids, training=True):
        """rows [len(ids), dim] for int ids (duplicates allowed); training pulls insert new keys"""
        ids = torch.as_tensor(ids, device=self.device).reshape(-1).long()
        uniq, inv = torch.unique(ids, return_inverse=True)
        if self.world == 1:
            return self._gather(uniq, training)[inv]
        keys_in, recv, order, send = self._route(uniq)
        vals_in = self._gather(keys_in, training)
        back = torch.empty(uniq.numel(), self.dim, dtype=torch.float32, device=self.device)
        tdist.all_to_all_single(back, vals_in.contiguous(), send.tolist(), recv.tolist(), group=self.group)
        vals = torch.empty_like(back)
        vals[order] = back
        return vals[inv]

    def push(self, ids, grads):
        """AdaGrad on the rows of ``ids`` with the summed gradient of duplicate ids"""
        ids = torch.as_tensor(ids, device=self.device).reshape(-1).long()
        grads = torch.as_tensor(grads, device=self.device).reshape(ids.numel(), self.dim).float()
        uniq, inv = torch.unique(ids, return_inverse=True)
        g = torch.zeros(uniq.numel(), self.dim, dtype=torch.float32, device=self.device).index_add_(0, inv, grads)
        if self.world == 1:
            self._update(uniq, g)
            return
        keys_in, recv, order, send = self._route(uniq)
        g_in = torch.empty(keys_in.numel(), self.dim, dtype=torch.float32, device=self.device)
        tdist.all_to_all_single(g_in, g[order].contiguous(), recv.tolist(), send.tolist(), group=self.group)
        self._update(keys_in, g_in)

    def local_size(self):
        return min(int(self.next_row.item()), self.max_rows) if self.gpu else len(self._map)

    def size(self):
        n = torch.tensor([self.local_size()], dtype=torch.int64)
        if self.world > 1:
            n = n.to(self.device) if self.gpu else n
            tdist.all_reduce(n, group=self.group)
        return int(n.item())

    def state_dict(self):
        """this rank's shard: {"keys": int64 [n], "values": float32 [n, dim], "g2sum": [n]}"""
        if self.gpu:
            live = (self.keys != _EMPTY) & (self.keys != _TOMB) & (self.rows >= 0)
            keys, rows = self.keys[live], self.rows[live].long()
        else:
            keys = torch.tensor(list(self._map.keys()), dtype=torch.int64)
            rows = torch.tensor(list(self._map.values()), dtype=torch.long)
        return {"keys": keys.cpu(), "values": self.W[rows].cpu(), "g2sum": self.g2[rows].cpu()}

    def set_state_dict(self, sd):
        keys = sd["keys"].to(self.device)
        rows = self._find(keys, True).long()
        self.W[rows] = sd["values"].to(self.device)
        self.g2[rows] = sd["g2sum"].to(self.device)


class _PullPushGpu(torch.autograd.Function):
    @staticmethod
    def forward(ctx, anchor, table, ids):
        ctx.table, ctx.ids = table, ids
        return table.pull(ids, training=True).reshape(*ids.shape, table.dim)

    @staticmethod
    def backward(ctx, gout):
        ctx.table.push(ctx.ids, gout.reshape(-1, ctx.table.dim))
        return gout.new_zeros(()), None, None


def _layer():
    from ...nn.layer.layers import Layer
    return Layer


class GpuPsEmbedding(_layer()):
    """Embedding whose table is a sharded HBM GpuPsTable (no dense [vocab, dim] parameter): the
    forward pulls, the backward pushes (the table's AdaGrad is the optimizer of these rows)."""

    def __init__(self, dim, max_rows_per_rank, **table_kw):
        super().__init__()
        self.table = GpuPsTable(dim, max_rows_per_rank, **table_kw)
        self._anchor = torch.zeros((), requires_grad=True)

    def forward(self, ids):
        t = ids._t if isinstance(ids, Tensor) else torch.as_tensor(ids)
        out = _PullPushGpu.apply(self._anchor, self.table, t.to(self.table.device).long())
        return _wrap(out)
