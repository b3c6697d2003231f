"""Fleet executor: run a task graph of micro-batch steps with credit-based flow control
(reference: paddle/fluid/distributed/fleet_executor/{fleet_executor,carrier,interceptor,
compute_interceptor,amplifier_interceptor,source_interceptor,sink_interceptor,task_node}.cc and
python/paddle/distributed/fleet/fleet_executor_utils.py TaskNode).

The scheduler is native (``csrc/runtime/fleet_executor.cpp``: one thread per local task, a step
starts when its upstreams produced it and every downstream edge still has buffer credit). Task
bodies are host callbacks: a ``Compute`` task runs a stage function or a static Program on its
upstreams' outputs for that micro-batch, ``Source`` produces micro-batches, ``Sink`` collects
results, ``Amplifier`` fires once every ``amplify`` upstream steps. An edge between tasks on
different ranks becomes a send task on the producer's rank and a recv task on the consumer's
(torch.distributed point-to-point: RCCL over xGMI on the GPU), so a pipeline's stages on
different GPUs overlap their compute with the activation transfers.
"""
from __future__ import annotations

import ctypes
import threading

import torch
import torch.distributed as tdist

from ..utils import native

__all__ = ["TaskNode", "FleetExecutor"]

_STEP_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_int, ctypes.c_int64, ctypes.c_void_p)
_ids = iter(range(1 << 30))


def _lib():
    L = native.lib()
    if not getattr(L, "_fe_sig", False):
        L.pha_fe_create.restype = ctypes.c_void_p
        L.pha_fe_destroy.argtypes = [ctypes.c_void_p]
        L.pha_fe_add_task.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.pha_fe_add_edge.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.pha_fe_run.argtypes = [ctypes.c_void_p, _STEP_FN, ctypes.c_void_p]
        L.pha_fe_trace_len.argtypes = [ctypes.c_void_p]
        L.pha_fe_trace_len.restype = ctypes.c_int64
        L.pha_fe_trace.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L._fe_sig = True
    return L


class TaskNode:
    """One task of the graph. ``fn(step, *upstream_outputs)`` is the body of a Compute / Sink /
    Amplifier task (a Source's ``fn(step)`` makes micro-batch ``step``); or pass a static
    ``program`` with ``feed_names`` (one per upstream, in add order) and ``fetch_list``."""

    def __init__(self, rank=0, max_run_times=1, role=None, program=None, task_id=None, node_type="Compute",
                 fn=None, amplify=1, feed_names=None, fetch_list=None, max_slot_nums=None, lazy_initialize=False):
        self.rank = int(rank)
        self.max_run_times = int(max_run_times)
        self.role = role
        self.program = program
        self._id = int(task_id) if task_id is not None else next(_ids) + 100000
        self.type = node_type
        self.fn = fn
        self.amplify = int(amplify)
        self.feed_names = list(feed_names or [])
        self.fetch_list = list(fetch_list or [])
        self.upstreams, self.downstreams = [], []

    def task_id(self):
        return self._id

    def add_upstream_task(self, upstream, buffer_size=2):
        self.upstreams.append((int(upstream), int(buffer_size)))

    def add_downstream_task(self, downstream, buffer_size=2):
        self.downstreams.append((int(downstream), int(buffer_size)))

    def set_type(self, t):
        self.type = t

    def set_run_pre_steps(self, n):
        self.max_run_times = int(n)

    def _run(self, step, inputs):
        if self.fn is not None:
            return self.fn(step, *inputs)
        if self.program is not None:
            from ..static import Executor
            feed = {n: v for n, v in zip(self.feed_names, inputs)}
            outs = Executor().run(self.program, feed=feed, fetch_list=self.fetch_list, return_numpy=False)
            return outs[0] if len(outs) == 1 else tuple(outs)
        return inputs[0] if len(inputs) == 1 else tuple(inputs)


def _meta(t):
    return torch.tensor([t.dim()] + list(t.shape) + [{torch.float32: 0, torch.float16: 1, torch.bfloat16: 2,
                                                     torch.int64: 3, torch.int32: 4}[t.dtype]], dtype=torch.int64)


_DTYPES = [torch.float32, torch.float16, torch.bfloat16, torch.int64, torch.int32]


class FleetExecutor:
    """Carrier of this rank: the tasks mapped to it (``task_id_to_rank``) plus a send / recv task
    per cross-rank edge. ``run()`` returns ``{sink task id: [result of each step]}``."""

    def __init__(self, exe_desc=None):
        self.exe_desc = exe_desc
        self._tasks = {}
        self.trace = []

    def init(self, carrier_id=None, program_desc=None, scope=None, place=None, num_micro_batches=1, task_nodes=None,
             task_id_to_rank=None, inference_root_scope_vars=None, fetch_var_names=None, group=None):
        self.num_micro_batches = int(num_micro_batches)
        self.task_nodes = {t.task_id(): t for t in task_nodes or []}
        self.task_id_to_rank = dict(task_id_to_rank or {t.task_id(): t.rank for t in task_nodes or []})
        self.group = group
        self.rank = tdist.get_rank(group) if tdist.is_available() and tdist.is_initialized() else 0
        return self

    def run(self, carrier_id=None):
        L = _lib()
        h = L.pha_fe_create()
        try:
            return self._run(L, h)
        finally:
            L.pha_fe_destroy(h)

    def _run(self, L, h):
        mine = {i: t for i, t in self.task_nodes.items() if self.task_id_to_rank.get(i, t.rank) == self.rank}
        bodies, ups_of, slots, results = {}, {}, {}, {}
        lock = threading.Lock()
        errors = []
        next_tid = [max(list(self.task_nodes) + [0]) + 1]

        def new_id():
            next_tid[0] += 1
            return next_tid[0]

        def add(tid, max_run, amplify=1):
            if L.pha_fe_add_task(h, tid, max_run, amplify) != 0:
                raise ValueError(f"bad task {tid}")

        for tid, t in mine.items():
            add(tid, t.max_run_times, t.amplify)
            bodies[tid] = t
            ups_of[tid] = []
        for tid, t in mine.items():
            for up, buff in t.upstreams:
                up_rank = self.task_id_to_rank.get(up, self.task_nodes[up].rank if up in self.task_nodes else self.rank)
                if up_rank == self.rank:
                    if L.pha_fe_add_edge(h, up, tid, max(buff, t.amplify)) != 0:
                        raise ValueError(f"bad edge {up}->{tid}")
                    ups_of[tid].append(up)
                else:   # recv task: pulls the remote upstream's output of each step
                    rid = new_id()
                    add(rid, self.task_nodes[up].max_run_times)
                    bodies[rid] = ("recv", up_rank)
                    ups_of[rid] = []
                    L.pha_fe_add_edge(h, rid, tid, max(buff, t.amplify))
                    ups_of[tid].append(rid)
            for down, buff in t.downstreams:
                d_rank = self.task_id_to_rank.get(down, self.task_nodes[down].rank if down in self.task_nodes
                                                  else self.rank)
                if d_rank != self.rank:   # send task: pushes each step's output to the remote consumer
                    sid = new_id()
                    add(sid, t.max_run_times)
                    bodies[sid] = ("send", d_rank)
                    ups_of[sid] = [tid]
                    L.pha_fe_add_edge(h, tid, sid, buff)

        n_down = {}
        for tid, ups in ups_of.items():
            for u in ups:
                n_down[u] = n_down.get(u, 0) + 1

        def take(u, step):
            with lock:
                key = (u, step)
                val, left = slots[key]
                if left <= 1:
                    del slots[key]
                else:
                    slots[key] = (val, left - 1)
            return val

        def body(tid, step, _ctx):
            try:
                b = bodies[tid]
                if isinstance(b, tuple) and b[0] == "send":
                    val = take(ups_of[tid][0], step)
                    ts = list(val) if isinstance(val, (tuple, list)) else [val]
                    tdist.send(torch.tensor([len(ts)], dtype=torch.int64), b[1], group=self.group)
                    for x in ts:
                        x = x._t if hasattr(x, "_t") else torch.as_tensor(x)
                        m = _meta(x)
                        tdist.send(torch.tensor([m.numel()], dtype=torch.int64), b[1], group=self.group)
                        tdist.send(m, b[1], group=self.group)
                        tdist.send(x.contiguous(), b[1], group=self.group)
                    out = None
                elif isinstance(b, tuple) and b[0] == "recv":
                    n = torch.zeros(1, dtype=torch.int64)
                    tdist.recv(n, b[1], group=self.group)
                    ts = []
                    for _ in range(int(n.item())):
                        ml = torch.zeros(1, dtype=torch.int64)
                        tdist.recv(ml, b[1], group=self.group)
                        m = torch.zeros(int(ml.item()), dtype=torch.int64)
                        tdist.recv(m, b[1], group=self.group)
                        nd = int(m[0])
                        buf = torch.empty([int(v) for v in m[1:1 + nd]], dtype=_DTYPES[int(m[-1])])
                        tdist.recv(buf, b[1], group=self.group)
                        ts.append(buf)
                    out = ts[0] if len(ts) == 1 else tuple(ts)
                else:
                    t = b
                    if t.amplify > 1:   # the amplifier reads the `amplify` upstream steps it covers
                        ins = [[take(u, s) for s in range(step * t.amplify, (step + 1) * t.amplify)]
                               for u in ups_of[tid]]
                    else:
                        ins = [take(u, step) for u in ups_of[tid]]
                    out = t._run(step, ins)
                    if t.type == "Sink" or not n_down.get(tid):
                        with lock:
                            results.setdefault(tid, []).append(out)
                if n_down.get(tid):
                    with lock:
                        slots[(tid, step)] = (out, n_down[tid])
                return 0
            except Exception as e:   # surfaced after the carrier stops
                errors.append(e)
                return -2

        cb = _STEP_FN(body)
        rc = L.pha_fe_run(h, cb, None)
        n = L.pha_fe_trace_len(h)
        tk = (ctypes.c_int32 * max(1, n))()
        st = (ctypes.c_int64 * max(1, n))()
        L.pha_fe_trace(h, tk, st)
        self.trace = [(tk[i], st[i]) for i in range(n)]
        if errors:
            raise errors[0]
        if rc != 0:
            raise RuntimeError(f"fleet executor failed ({rc})")
        return {k: v for k, v in results.items() if k in self.task_nodes}
