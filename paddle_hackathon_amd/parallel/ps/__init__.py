"""Parameter-server training (``paddle.distributed.ps``; reference:
python/paddle/distributed/ps/the_one_ps.py (TheOnePSRuntime: _init_server/_run_server/
_init_worker/_stop_worker/_save_persistables/_shrink), paddle/fluid/distributed/ps/{service,table},
python/paddle/distributed/entry_attr.py, python/paddle/fluid/contrib/layers/nn.py:sparse_embedding).

The tables live in a native C++ server (``csrc/runtime/ps.cpp``): dense tables (one flat float32
vector, server-side SGD / AdaGrad / Adam, optional synchronous merge of all trainers' gradients)
and sparse tables (id -> row hash shards created on first training pull, admission by
``ProbabilityEntry`` / ``CountFilterEntry``, the reference's Naive / AdaGrad / StdAdaGrad / Adam
sparse rules). Trainers are ordinary GPU processes: dense parameters stay in HBM and are synced
through the server once per step by :class:`PSOptimizer`; embedding rows are pulled for the
unique ids of a batch, copied to the device, and their summed gradients pushed back in backward
(:class:`DistributedEmbedding`). Dense tables are split into contiguous chunks over the servers,
sparse ids are routed by ``id % n_servers``.

Modes (``DistributedStrategy.a_sync`` / ``a_sync_configs["k_steps"]`` as in the reference):
``sync`` (a_sync False: every dense push is merged over all trainers and applied once; pulls wait
for that version), ``async`` (a_sync True, k_steps <= 0: each push is applied on arrival) and
``geo`` (k_steps > 0: trainers step locally and every k steps push their parameter delta).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from ...utils import native

__all__ = ["PSServer", "PSClient", "DistributedEmbedding", "PSOptimizer", "TheOnePSRuntime", "RULES",
           "sparse_embedding", "GpuPsTable", "GpuPsEmbedding"]

RULES = {"sgd": 0, "naive": 0, "adagrad": 1, "std_adagrad": 2, "adam": 3, "sum": 4, "ctr": 5}

# CtrCommonAccessor defaults (reference ps/table/ctr_accessor.cc + the_one_ps.py accessor config)
CTR_DEFAULTS = {"nonclk_coeff": 0.1, "click_coeff": 1.0, "embedx_threshold": 10.0, "show_click_decay_rate": 0.98,
                "delete_threshold": 0.8, "delete_after_unseen_days": 30.0, "base_threshold": 1.5}

_P = ctypes.c_void_p
_sigs_done = False


def _lib():
    global _sigs_done
    L = native.lib()
    if not _sigs_done:
        i64, u32, u64, i32 = ctypes.c_int64, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
        sig = {
            "pha_ps_server_start": (_P, [ctypes.c_char_p, i32]),
            "pha_ps_server_port": (i32, [_P]),
            "pha_ps_server_wait": (i32, [_P, i64]),
            "pha_ps_server_destroy": (None, [_P]),
            "pha_ps_client_connect": (_P, [ctypes.c_char_p, i32, i64]),
            "pha_ps_client_close": (None, [_P]),
            "pha_ps_create_dense": (i64, [_P, u32, u64, _P, _P, _P]),
            "pha_ps_create_sparse": (i64, [_P, u32, _P, _P, u64]),
            "pha_ps_set_dense": (i64, [_P, u32, _P, u64]),
            "pha_ps_pull_dense": (i64, [_P, u32, _P, u64, u32]),
            "pha_ps_push_dense": (i64, [_P, u32, _P, u64]),
            "pha_ps_pull_sparse": (i64, [_P, u32, _P, u64, i32, _P, i32]),
            "pha_ps_push_sparse": (i64, [_P, u32, _P, u64, i32, _P, i32]),
            "pha_ps_barrier": (i64, [_P, u32, u64]),
            "pha_ps_table_size": (i64, [_P, u32]),
            "pha_ps_shrink": (i64, [_P, u32, u32]),
            "pha_ps_save": (i64, [_P, u32, ctypes.c_char_p, i32, i32]),
            "pha_ps_stop_server": (i64, [_P]),
            "pha_ps_set_spill": (i64, [_P, u32, ctypes.c_char_p]),
            "pha_ps_graph_add_edges": (i64, [_P, u32, _P, _P, _P, u64, i32]),
            "pha_ps_graph_sample": (i64, [_P, u32, _P, u64, u32, i32, _P, u64]),
            "pha_ps_graph_feat": (i64, [_P, u32, _P, u64, u32, _P, i32]),
            "pha_ps_graph_random_nodes": (i64, [_P, u32, u32, u64, _P]),
            "pha_ps_graph_node_count": (i64, [_P, u32]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _sigs_done = True
    return L


def _ok(rc, what):
    if rc < 0:
        raise RuntimeError(f"parameter server {what} failed (status {rc})")
    return rc


def _a(x, dt):
    return np.ascontiguousarray(x, dtype=dt)


def _split_endpoint(ep):
    host, port = ep.rsplit(":", 1)
    return host, int(port)


class PSServer:
    """One parameter-server process' tables, served on ``host:port`` (port 0 = pick a free one)."""

    def __init__(self, host="0.0.0.0", port=0):
        self._h = _lib().pha_ps_server_start(host.encode(), int(port))
        if not self._h:
            raise OSError(f"cannot listen on {host}:{port}")

    @property
    def port(self):
        return _lib().pha_ps_server_port(self._h)

    def run(self, timeout=None):
        """Block until a trainer stops the server (``PSClient.stop_servers``); True if stopped."""
        return bool(_lib().pha_ps_server_wait(self._h, -1 if timeout is None else int(timeout * 1000)))

    def stop(self):
        if self._h:
            _lib().pha_ps_server_destroy(self._h)
            self._h = None

    def __del__(self):
        if getattr(self, "_h", None) and native._lib is not None:
            self.stop()


def _entry_cfg(entry):
    """(entry_kind, entry_value) from a ProbabilityEntry / CountFilterEntry (or None)."""
    if entry is None:
        return 0, 0.0
    name = type(entry).__name__
    args = getattr(entry, "args", ())
    if name == "ProbabilityEntry":
        return 1, float(args[0] if args else getattr(entry, "_probability", 1.0))
    if name == "CountFilterEntry":
        return 2, float(args[0] if args else getattr(entry, "_count_filter", 0))
    return 0, 0.0


class PSClient:
    """Connections to every server of the job (``endpoints``: list of "ip:port")."""

    def __init__(self, endpoints, timeout=60.0):
        L = _lib()
        self.endpoints = list(endpoints)
        self._h = []
        for ep in self.endpoints:
            host, port = _split_endpoint(ep)
            h = L.pha_ps_client_connect(host.encode(), port, int(timeout * 1000))
            if not h:
                self.close()
                raise ConnectionError(f"no parameter server at {ep} after {timeout}s")
            self._h.append(h)
        self._dense = {}    # table -> (numel, chunk bounds)
        self._sparse = {}   # table -> dim

    @property
    def n_servers(self):
        return len(self._h)

    def close(self):
        L = _lib()
        for h in self._h:
            L.pha_ps_client_close(h)
        self._h = []

    def _bounds(self, numel):
        n = self.n_servers
        per, extra = divmod(numel, n)
        b, off = [], 0
        for i in range(n):
            size = per + (1 if i < extra else 0)
            b.append((off, off + size))
            off += size
        return b

    @staticmethod
    def _cfg(rule, dim, sync_trainers, entry, lr, beta1, beta2, epsilon, initial_g2sum, initial_range, bounds,
             ctr=None, cache_rows=0):
        kind, value = _entry_cfg(entry)
        iv = _a([RULES[rule] if isinstance(rule, str) else int(rule), dim, sync_trainers, kind, int(cache_rows)],
                np.int32)
        lo, hi = bounds if bounds is not None else (-3.4e38, 3.4e38)
        c = dict(CTR_DEFAULTS, **(ctr or {}))
        fv = _a([lr, beta1, beta2, epsilon, initial_g2sum, initial_range, lo, hi, value, c["nonclk_coeff"],
                 c["click_coeff"], c["embedx_threshold"], c["show_click_decay_rate"], c["delete_threshold"],
                 c["delete_after_unseen_days"], c["base_threshold"]], np.float32)
        return iv, fv

    # ---- dense -------------------------------------------------------------------------
    def create_dense(self, table, numel, rule="sgd", lr=0.01, init=None, sync_trainers=1, beta1=0.9, beta2=0.999,
                     epsilon=1e-8, initial_g2sum=3.0, bounds=None):
        iv, fv = self._cfg(rule, 1, sync_trainers, None, lr, beta1, beta2, epsilon, initial_g2sum, 0.0, bounds)
        init = None if init is None else _a(init, np.float32).reshape(-1)
        L = _lib()
        bounds_ = self._bounds(int(numel))
        for h, (s, e) in zip(self._h, bounds_):
            p = init[s:e].ctypes.data if init is not None else None
            _ok(L.pha_ps_create_dense(h, table, e - s, iv.ctypes.data, fv.ctypes.data, p), "create_dense")
        self._dense[table] = (int(numel), bounds_)

    def _dense_info(self, table):
        if table not in self._dense:
            raise KeyError(f"dense table {table} not created by this client")
        return self._dense[table]

    def set_dense(self, table, values):
        numel, b = self._dense_info(table)
        v = _a(values, np.float32).reshape(-1)
        for h, (s, e) in zip(self._h, b):
            _ok(_lib().pha_ps_set_dense(h, table, v[s:e].ctypes.data, e - s), "set_dense")

    def pull_dense(self, table, out=None, min_version=0):
        numel, b = self._dense_info(table)
        out = np.empty(numel, np.float32) if out is None else out
        for h, (s, e) in zip(self._h, b):
            _ok(_lib().pha_ps_pull_dense(h, table, out[s:e].ctypes.data, e - s, int(min_version)), "pull_dense")
        return out

    def push_dense(self, table, grad):
        """Returns the table version after the push (sync mode: the merged version)."""
        numel, b = self._dense_info(table)
        g = _a(grad, np.float32).reshape(-1)
        if g.size != numel:
            raise ValueError(f"dense table {table} has {numel} elements, got {g.size}")
        ver = 0
        for h, (s, e) in zip(self._h, b):
            ver = _ok(_lib().pha_ps_push_dense(h, table, g[s:e].ctypes.data, e - s), "push_dense")
        return ver

    # ---- sparse ------------------------------------------------------------------------
    def create_sparse(self, table, dim, rule="adagrad", lr=0.05, initial_range=1e-4, entry=None, seed=0,
                      beta1=0.9, beta2=0.999, epsilon=1e-8, initial_g2sum=3.0, bounds=(-10.0, 10.0), accessor=None,
                      ctr_config=None, cache_rows=0, spill_dir=None):
        """``accessor="ctr"``: CtrCommonAccessor rows — pulls return [embed_w, embedx(dim-1)], pushes
        carry [show, click, grads] (``push_sparse_ctr``); embedx is created once the feature's score
        (show-click)*nonclk_coeff + click*click_coeff reaches ``embedx_threshold``.
        ``cache_rows`` + ``spill_dir``: SSD-table mode, at most ``cache_rows`` rows resident per
        server, colder rows spilled to files under ``spill_dir`` and read back on access."""
        if accessor == "ctr":
            rule = "ctr"
        iv, fv = self._cfg(rule, dim, 1, entry, lr, beta1, beta2, epsilon, initial_g2sum, initial_range, bounds,
                           ctr_config, cache_rows)
        for h in self._h:
            _ok(_lib().pha_ps_create_sparse(h, table, iv.ctypes.data, fv.ctypes.data, int(seed)), "create_sparse")
            if cache_rows and spill_dir:
                os.makedirs(spill_dir, exist_ok=True)
                _ok(_lib().pha_ps_set_spill(h, table, os.path.abspath(spill_dir).encode()), "set_spill")
        self._sparse[table] = int(dim)
        self._ctr = getattr(self, "_ctr", set())
        if rule == "ctr":
            self._ctr.add(table)

    def _route(self, ids):
        ids = _a(ids, np.uint64).reshape(-1)
        srv = (ids % np.uint64(self.n_servers)).astype(np.int64)
        return ids, srv

    def pull_sparse(self, table, ids, training=True):
        """Rows [len(ids), dim] (float32) for ``ids`` (any int array, duplicates allowed)."""
        dim = self._sparse[table]
        ids, srv = self._route(ids)
        out = np.empty((ids.size, dim), np.float32)
        L = _lib()
        for i, h in enumerate(self._h):
            sel = np.nonzero(srv == i)[0]
            if sel.size == 0:
                continue
            sub_ids = np.ascontiguousarray(ids[sel])
            buf = np.empty((sel.size, dim), np.float32)
            _ok(L.pha_ps_pull_sparse(h, table, sub_ids.ctypes.data, sel.size, dim, buf.ctypes.data, int(training)),
                "pull_sparse")
            out[sel] = buf
        return out

    def push_sparse(self, table, ids, grads, delta=False):
        dim = self._sparse[table]
        ids, srv = self._route(ids)
        g = _a(grads, np.float32).reshape(ids.size, dim)
        L = _lib()
        for i, h in enumerate(self._h):
            sel = np.nonzero(srv == i)[0]
            if sel.size == 0:
                continue
            sub_ids = np.ascontiguousarray(ids[sel])
            sub_g = np.ascontiguousarray(g[sel])
            _ok(L.pha_ps_push_sparse(h, table, sub_ids.ctypes.data, sel.size, dim, sub_g.ctypes.data, int(delta)),
                "push_sparse")

    def push_sparse_ctr(self, table, ids, shows, clicks, grads):
        """CTR accessor push: per id its show / click counts and the gradient of [embed, embedx]"""
        dim = self._sparse[table]
        ids, srv = self._route(ids)
        g = _a(grads, np.float32).reshape(ids.size, dim)
        payload = np.concatenate([_a(shows, np.float32).reshape(-1, 1), _a(clicks, np.float32).reshape(-1, 1), g], 1)
        L = _lib()
        for i, h in enumerate(self._h):
            sel = np.nonzero(srv == i)[0]
            if sel.size == 0:
                continue
            sub_ids = np.ascontiguousarray(ids[sel])
            sub = np.ascontiguousarray(payload[sel])
            _ok(L.pha_ps_push_sparse(h, table, sub_ids.ctypes.data, sel.size, dim + 2, sub.ctypes.data, 0),
                "push_sparse_ctr")

    # ---- graph table (common_graph_table) ------------------------------------------------
    def _graph_route(self, ids):
        ids = _a(ids, np.uint64).reshape(-1)
        return ids, (ids % np.uint64(self.n_servers)).astype(np.int64)

    def graph_add_edges(self, table, src, dst, weight=None, bidirectional=False):
        """edges live on the server of their source node"""
        src = _a(src, np.uint64).reshape(-1)
        dst = _a(dst, np.uint64).reshape(-1)
        w = _a(np.ones(src.size) if weight is None else weight, np.float32).reshape(-1)
        passes = [(src, dst)] + ([(dst, src)] if bidirectional else [])
        L = _lib()
        for a, b in passes:
            srv = (a % np.uint64(self.n_servers)).astype(np.int64)
            for i, h in enumerate(self._h):
                sel = np.nonzero(srv == i)[0]
                if sel.size:   # keep the contiguous copies alive across the native call
                    sa, sb, sw = (np.ascontiguousarray(v[sel]) for v in (a, b, w))
                    _ok(L.pha_ps_graph_add_edges(h, table, sa.ctypes.data, sb.ctypes.data, sw.ctypes.data, sel.size,
                                                 0), "graph_add")
        # every endpoint is a node on its own server (sink nodes are sampled / counted too)
        nodes = np.unique(np.concatenate([src, dst]))
        srv = (nodes % np.uint64(self.n_servers)).astype(np.int64)
        for i, h in enumerate(self._h):
            sel = np.nonzero(srv == i)[0]
            if sel.size:
                sub = np.ascontiguousarray(nodes[sel])
                _ok(L.pha_ps_graph_add_edges(h, table, sub.ctypes.data, None, None, sel.size, 2), "graph_nodes")

    def graph_sample_neighbors(self, table, ids, sample_size, weighted=False):
        """-> list (one per id) of sampled neighbour id arrays (<= sample_size, without replacement)"""
        ids, srv = self._graph_route(ids)
        res = [None] * ids.size
        L = _lib()
        for i, h in enumerate(self._h):
            sel = np.nonzero(srv == i)[0]
            if sel.size == 0:
                continue
            sub = np.ascontiguousarray(ids[sel])
            cap = sel.size * 4 + sel.size * int(sample_size) * 8
            buf = np.empty(cap, np.uint8)
            nb = _ok(L.pha_ps_graph_sample(h, table, sub.ctypes.data, sel.size, int(sample_size), int(weighted),
                                           buf.ctypes.data, cap), "graph_sample")
            counts = buf[:sel.size * 4].view(np.uint32)
            picked = buf[sel.size * 4:nb].view(np.uint64)
            off = 0
            for j, c in zip(sel, counts):
                res[j] = picked[off:off + c].astype(np.int64)
                off += int(c)
        return res

    def graph_set_node_feat(self, table, ids, feats):
        ids, srv = self._graph_route(ids)
        f = _a(feats, np.float32).reshape(ids.size, -1)
        for i, h in enumerate(self._h):
            sel = np.nonzero(srv == i)[0]
            if sel.size:
                sub_f = np.ascontiguousarray(f[sel])
                sub_i = np.ascontiguousarray(ids[sel])
                _ok(_lib().pha_ps_graph_feat(h, table, sub_i.ctypes.data, sel.size, f.shape[1], sub_f.ctypes.data, 1),
                    "graph_set_feat")

    def graph_get_node_feat(self, table, ids, dim):
        ids, srv = self._graph_route(ids)
        out = np.zeros((ids.size, dim), np.float32)
        for i, h in enumerate(self._h):
            sel = np.nonzero(srv == i)[0]
            if sel.size:
                buf = np.empty((sel.size, dim), np.float32)
                sub_i = np.ascontiguousarray(ids[sel])
                _ok(_lib().pha_ps_graph_feat(h, table, sub_i.ctypes.data, sel.size, dim, buf.ctypes.data, 0),
                    "graph_get_feat")
                out[sel] = buf
        return out

    def graph_random_sample_nodes(self, table, k, seed=0):
        out = []
        per = [k // self.n_servers + (1 if i < k % self.n_servers else 0) for i in range(self.n_servers)]
        for h, n in zip(self._h, per):
            if n:
                buf = np.empty(n, np.uint64)
                got = _ok(_lib().pha_ps_graph_random_nodes(h, table, n, int(seed), buf.ctypes.data), "graph_random")
                out.append(buf[:got])
        return np.concatenate(out).astype(np.int64) if out else np.zeros(0, np.int64)

    def graph_node_count(self, table):
        return sum(_ok(_lib().pha_ps_graph_node_count(h, table), "graph_count") for h in self._h)

    # ---- control -----------------------------------------------------------------------
    def barrier(self, n, tag=0):
        """Block until ``n`` trainers reached barrier ``tag`` (served by the first server)."""
        _ok(_lib().pha_ps_barrier(self._h[0], int(tag), int(n)), "barrier")

    def table_size(self, table):
        return sum(_ok(_lib().pha_ps_table_size(h, table), "table_size") for h in self._h) if table in self._sparse \
            else self._dense_info(table)[0]

    def shrink(self, table, max_idle=0):
        """Drop sparse rows not pulled since the last ``max_idle`` shrink passes; returns rows dropped."""
        return sum(_ok(_lib().pha_ps_shrink(h, table, int(max_idle)), "shrink") for h in self._h)

    def _files(self, table, dirname):
        return [os.path.join(dirname, f"table_{table}.shard{i}") for i in range(self.n_servers)]

    def save(self, table, dirname, mode=0):
        """mode 0: weights + optimizer state; mode 1: weights only (inference)."""
        os.makedirs(dirname, exist_ok=True)
        for h, f in zip(self._h, self._files(table, dirname)):
            _ok(_lib().pha_ps_save(h, table, os.path.abspath(f).encode(), int(mode), 0), "save")

    def load(self, table, dirname):
        for h, f in zip(self._h, self._files(table, dirname)):
            _ok(_lib().pha_ps_save(h, table, os.path.abspath(f).encode(), 0, 1), "load")

    def stop_servers(self):
        for h in self._h:
            _lib().pha_ps_stop_server(h)

    def __del__(self):
        if getattr(self, "_h", None) and native._lib is not None:
            self.close()


# ---------------------------------------------------------------------------------- runtime
class TheOnePSRuntime:
    """Role-aware glue used by ``fleet`` in parameter-server mode."""

    def __init__(self, role_maker, strategy):
        self.role_maker = role_maker
        self.strategy = strategy
        self.server = None
        self.client = None
        self._next_table = 0

    # server side
    def init_server(self, dirname=None, var_names=None, **kwargs):
        host, port = _split_endpoint(self.role_maker._get_pserver_endpoints()[self.role_maker._server_index()])
        self.server = PSServer("0.0.0.0", port)
        self._load_dir = dirname

    def run_server(self):
        if self.server is None:
            self.init_server()
        self.server.run()
        self.server.stop()
        self.server = None

    # trainer side
    def init_worker(self, scopes=None):
        self.client = PSClient(self.role_maker._get_pserver_endpoints())

    def new_table_id(self):
        t = self._next_table
        self._next_table += 1
        return t

    def barrier_worker(self):
        if self.client is not None:
            self.client.barrier(self.role_maker._worker_num(), tag=1 << 20)

    def stop_worker(self):
        if self.client is None:
            return
        self.barrier_worker()
        if self.role_maker._worker_index() == 0:
            self.client.stop_servers()
        self.client.close()
        self.client = None

    def mode(self):
        if not self.strategy.a_sync:
            return "sync"
        k = int(self.strategy.a_sync_configs.get("k_steps", -1))
        return "geo" if k > 0 else "async"


_runtime = None


def set_runtime(rt):
    global _runtime
    _runtime = rt


def get_runtime():
    if _runtime is None or _runtime.client is None:
        raise RuntimeError("parameter-server mode needs fleet.init(role_maker) and fleet.init_worker() first")
    return _runtime


# -------------------------------------------------------------------------------- trainer ops
class _PullPush(torch.autograd.Function):
    """Forward: rows of the batch's unique ids (pulled by the caller); backward: sum the output
    gradient per unique id and push it to the sparse table."""

    @staticmethod
    def forward(ctx, rows, inverse, anchor, client, table, uniq, padding_idx):
        ctx.save_for_backward(inverse)
        ctx.meta = (client, table, uniq, padding_idx, rows.shape[0])
        return rows.index_select(0, inverse.reshape(-1)).reshape(*inverse.shape, rows.shape[1])

    @staticmethod
    def backward(ctx, gout):
        (inverse,) = ctx.saved_tensors
        client, table, uniq, padding_idx, n = ctx.meta
        g = torch.zeros(n, gout.shape[-1], dtype=torch.float32, device=gout.device)
        g.index_add_(0, inverse.reshape(-1), gout.reshape(-1, gout.shape[-1]).float())
        g = g.cpu().numpy()
        if padding_idx is not None:
            g[uniq == padding_idx] = 0.0
        client.push_sparse(table, uniq, g)
        return None, None, gout.new_zeros(()), None, None, None, None


def _layer_base():
    from ...nn.layer.layers import Layer
    return Layer


class DistributedEmbedding(_layer_base()):
    """Embedding whose rows live in a parameter-server sparse table (the dygraph form of the
    reference's ``sparse_embedding``). ``size = [vocab (unused: the table grows with the ids
    seen), dim]``. Rows of a batch's unique ids are pulled in forward (training pulls create
    rows that the entry policy admits); their summed gradients are pushed in backward and the
    server applies the sparse rule (``rule``: naive/sgd, adagrad, std_adagrad, adam)."""

    def __init__(self, size, padding_idx=None, entry=None, rule="adagrad", lr=0.05, initial_range=None,
                 table_id=None, is_test=False):
        super().__init__()
        self.dim = int(size[1])
        self.padding_idx = padding_idx
        self.entry = entry
        self.rule, self.lr = rule, lr
        self.initial_range = initial_range if initial_range is not None else 1.0 / np.sqrt(self.dim)
        self.table_id = table_id
        self.is_test = is_test
        self._created = False
        # scalar leaf (not a model parameter) that makes autograd reach the push in backward
        self._anchor = torch.zeros((), requires_grad=True)

    def _ensure(self):
        rt = get_runtime()
        if self.table_id is None:
            self.table_id = rt.new_table_id()
        if not self._created:
            rt.client.create_sparse(self.table_id, self.dim, rule=self.rule, lr=self.lr,
                                    initial_range=self.initial_range, entry=self.entry, seed=self.table_id + 1)
            self._created = True
        return rt.client

    def forward(self, ids):
        from ...framework.core import Tensor, _wrap
        t = ids._t if isinstance(ids, Tensor) else torch.as_tensor(ids)
        client = self._ensure()
        flat = t.detach().reshape(-1).cpu().numpy().astype(np.int64)
        uniq, inv = np.unique(flat, return_inverse=True)
        training = self.training and not self.is_test
        rows = client.pull_sparse(self.table_id, uniq, training=training)
        if self.padding_idx is not None:
            rows[uniq == self.padding_idx] = 0.0
        dev = t.device
        rows_t = torch.from_numpy(rows).to(dev, non_blocking=True)
        inv_t = torch.from_numpy(inv.reshape(t.shape)).to(dev)
        if not (training and torch.is_grad_enabled()):
            return _wrap(rows_t.index_select(0, inv_t.reshape(-1)).reshape(*t.shape, self.dim))
        out = _PullPush.apply(rows_t, inv_t, self._anchor, client, self.table_id, uniq, self.padding_idx)
        return _wrap(out)


def sparse_embedding(input, size, padding_idx=None, is_test=False, entry=None, table_class="MemorySparseTable",
                     param_attr=None, dtype="float32", slot=None):
    """Functional form of the reference's ``sparse_embedding`` (one layer per call site name)."""
    name = getattr(param_attr, "name", None) or f"sparse_embedding_{int(size[1])}"
    layer = _EMB_CACHE.get(name)
    if layer is None:
        layer = _EMB_CACHE[name] = DistributedEmbedding(size, padding_idx=padding_idx, entry=entry, is_test=is_test)
    return layer(input)


_EMB_CACHE = {}


class PSOptimizer:
    """Dense-parameter sync through the parameter server, wrapping a local optimizer.

    sync / async: the flattened fp32 gradient of every trainable parameter is pushed to one dense
    table whose server-side rule is the wrapped optimizer's (SGD / Adam / Adagrad); the updated
    parameters are pulled back (sync: after all trainers' gradients were merged and applied).
    geo: the local optimizer steps every iteration; every ``k_steps`` the parameter delta since
    the last sync is pushed (server adds it) and the merged parameters are pulled back.
    """

    def __init__(self, optimizer, runtime, strategy):
        self._inner_opt = optimizer
        self._rt = runtime
        self._mode = runtime.mode()
        self._k = max(1, int(strategy.a_sync_configs.get("k_steps", 1) or 1))
        self._params = [p for p in optimizer._parameter_list if not p.stop_gradient]
        self._table = None
        self._version = 0
        self._steps = 0
        self._base = None

    def _flat(self, tensors):
        return torch.cat([t.detach().reshape(-1).float() for t in tensors]).cpu().numpy()

    def _assign(self, flat):
        off = 0
        with torch.no_grad():
            for p in self._params:
                n = p._t.numel()
                p._t.copy_(torch.from_numpy(flat[off:off + n]).reshape(p._t.shape).to(p._t.device, p._t.dtype))
                off += n

    def _init_table(self):
        rt = self._rt
        opt = self._inner_opt
        name = type(opt).__name__.lower()
        rule = "sum" if self._mode == "geo" else ("adam" if "adam" in name else "adagrad" if "adagrad" in name else "sgd")
        lr = float(opt.get_lr()) if hasattr(opt, "get_lr") else 0.01
        init = self._flat([p._t for p in self._params])
        self._table = rt.new_table_id()
        ws = rt.role_maker._worker_num()
        rt.client.create_dense(self._table, init.size, rule=rule, lr=lr, init=init,
                               sync_trainers=ws if self._mode == "sync" else 1,
                               beta1=getattr(opt, "_beta1", 0.9), beta2=getattr(opt, "_beta2", 0.999),
                               epsilon=getattr(opt, "_epsilon", 1e-8))
        rt.barrier_worker()                       # every trainer sees the first creator's init
        self._assign(rt.client.pull_dense(self._table))
        self._base = rt.client.pull_dense(self._table) if self._mode == "geo" else None

    def step(self):
        if self._table is None:
            self._init_table()
        c = self._rt.client
        self._steps += 1
        if self._mode == "geo":
            self._inner_opt.step()
            if self._steps % self._k == 0:
                cur = self._flat([p._t for p in self._params])
                c.push_dense(self._table, (cur - self._base) / self._rt.role_maker._worker_num())
                self._base = c.pull_dense(self._table)
                self._assign(self._base)
            return
        grads = [p._t.grad if p._t.grad is not None else torch.zeros_like(p._t) for p in self._params]
        self._version = c.push_dense(self._table, self._flat(grads))
        if self._mode == "sync":
            self._version = self._steps   # the merged update of this step
        self._assign(c.pull_dense(self._table, min_version=self._version if self._mode == "sync" else 0))

    def minimize(self, loss, startup_program=None, parameters=None, no_grad_set=None):
        self.step()

    def clear_grad(self, set_to_zero=True):
        self._inner_opt.clear_grad(set_to_zero)

    def __getattr__(self, item):
        return getattr(self._inner_opt, item)


from .gpu_ps import GpuPsTable, GpuPsEmbedding  # noqa: E402,F401  (HBM-resident sharded tables)
