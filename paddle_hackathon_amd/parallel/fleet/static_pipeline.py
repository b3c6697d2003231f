"""Static-graph pipeline parallelism (reference: python/paddle/fluid/optimizer.py PipelineOptimizer,
distributed/fleet/meta_optimizers/pipeline_optimizer.py; the section program of each stage run by
paddle/fluid/framework/section_worker.cc).

Stages. Ops recorded under ``paddle.static.device_guard("gpu:k")`` carry ``op_device`` and belong
to stage k. After the per-op backward (static/backward.py) every grad op inherits the stage of
its forward op; ``sum`` / alias / zero-fill grad ops the stage of the variable whose gradient
they form; the loss-gradient seed the loss's stage. Every edge of the op graph that crosses a
stage boundary — an activation going forward, an activation gradient (or a shared parameter's
partial gradient) going backward — becomes a point-to-point transfer: the producing stage posts a
non-blocking send right after the producer op, the consuming stage receives right before the
first consumer. One rank runs one stage (rank = stage index within the pipeline group).

Schedule. ``Executor.run`` on a pipelined program splits the feed along the batch dimension into
``accumulate_steps`` micro-batches, runs every micro-batch's forward section, then every
micro-batch's backward section (GPipe order; all ranks walk the same op sequence; receives are
posted in each sender's send order — RCCL matches point-to-point messages by order, not tag — and
the non-blocking sends cannot deadlock), averages each parameter gradient over
the micro-batches and applies the inner optimizer to the stage's own parameters. Fetches of a
variable computed on this stage return the mean over micro-batches (None on other stages).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as tdist

from ...framework.core import Tensor, Parameter, _wrap
from ...static import program as P
from ...static import backward as B


def _stage_of_device(dev):
    if dev is None:
        return None
    s = str(dev)
    return int(s.rsplit(":", 1)[-1]) if ":" in s else 0


def assign_stages(prog):
    """-> {id(op): stage} for every op of the global block"""
    blk = prog.global_block()
    producer, stage = {}, {}
    first_reader = {}
    grad_of = prog.__dict__.get("_grad_of", {})
    by_name = {}
    for op in blk.ops:
        if B.op_role(op) == B.FORWARD:
            st = _stage_of_device(op.attrs.get("op_device"))
            if st is None:   # no device_guard: the stage of the first input's producer (else 0)
                st = 0
                for v in P._iter_vars((op.args, op.kwargs)):
                    if id(v) in producer:
                        st = stage[id(producer[id(v)])]
                        break
            stage[id(op)] = st
            for v in P._iter_tensors((op.args, op.kwargs)):
                if isinstance(v, Parameter):
                    first_reader.setdefault(id(v), st)
        for v in P._iter_vars(op.outputs):
            producer[id(v)] = op
            by_name[v.name] = v

    def var_stage(name):
        v = blk.vars.get(name)
        if v is not None and id(v) in producer and id(producer[id(v)]) in stage:
            return stage[id(producer[id(v)])]
        for p in prog.all_parameters():
            if p.name == name:
                return first_reader.get(id(p), 0)
        return 0

    for op in blk.ops:
        if id(op) in stage:
            continue
        fwd = grad_of.get(id(op))
        if fwd is not None and id(fwd) in stage:
            stage[id(op)] = stage[id(fwd)]
        elif B.op_role(op) == B.LOSS:
            x = op.kwargs.get("x")
            stage[id(op)] = stage.get(id(producer.get(id(x))), 0) if x is not None else 0
        elif op.attrs.get("op_role_var"):
            stage[id(op)] = var_stage(op.attrs["op_role_var"][0])
        else:
            stage[id(op)] = 0
    return stage, first_reader


_DT = [torch.float32, torch.float16, torch.bfloat16, torch.float64, torch.int64, torch.int32, torch.bool,
       torch.uint8, torch.int8]
_HDR = 10     # fixed header length: [ndim, dims (<= 8, zero padded), dtype]


class _Transfer:
    """a non-blocking send after a producer / a blocking receive before a consumer; each tensor
    travels as a fixed-size header [ndim, dims, dtype] and its data (two tags)"""

    def __init__(self, runner):
        self.r = runner
        self.pending = []

    def send(self, t, dst, tag):
        g = self.r.group
        t = t.detach().contiguous()
        if self.r.cpu_comm:
            t = t.cpu()
        hdr = torch.zeros(_HDR, dtype=torch.int64)
        hdr[0] = t.dim()
        hdr[1:1 + t.dim()] = torch.tensor(list(t.shape), dtype=torch.int64)
        hdr[-1] = _DT.index(t.dtype)
        if not self.r.cpu_comm:
            hdr = hdr.to(t.device)
        self.pending.append(tdist.isend(hdr, self.r.ranks[dst], group=g, tag=2 * tag))
        self.pending.append(tdist.isend(t, self.r.ranks[dst], group=g, tag=2 * tag + 1))
        self.pending.append((hdr, t))     # the buffers stay alive until wait()

    def recv(self, src, tag, device):
        g = self.r.group
        hdr = torch.zeros(_HDR, dtype=torch.int64, device="cpu" if self.r.cpu_comm else device)
        tdist.recv(hdr, self.r.ranks[src], group=g, tag=2 * tag)
        h = hdr.cpu().tolist()
        shape, dt = h[1:1 + h[0]], _DT[h[-1]]
        buf = torch.empty(shape, dtype=dt, device="cpu" if self.r.cpu_comm else device)
        tdist.recv(buf, self.r.ranks[src], group=g, tag=2 * tag + 1)
        return buf.to(device)

    def wait(self):
        for w in self.pending:
            if hasattr(w, "wait"):
                w.wait()
        self.pending = []


class PipelineRunner:
    def __init__(self, prog, optimizer, params_grads, n_stages, stage, micro_batches, ranks=None, group=None):
        self.prog, self.opt = prog, optimizer
        self.n_stages, self.stage, self.k = n_stages, stage, max(1, int(micro_batches))
        self.ranks = ranks or list(range(n_stages))
        self.group = group
        backend = tdist.get_backend(group) if tdist.is_initialized() else "gloo"
        self.cpu_comm = backend == "gloo"
        self.op_stage, self.param_stage = assign_stages(prog)
        blk = prog.global_block()
        self.fwd_ops = [op for op in blk.ops if B.op_role(op) in (B.FORWARD, B.LOSS)]
        self.bwd_ops = [op for op in blk.ops if B.op_role(op) == B.BACKWARD]
        self.params = [(p, g) for p, g in params_grads if self.param_stage.get(id(p), 0) == stage]
        if optimizer._parameter_list is None or set(map(id, optimizer._parameter_list)) != {id(p) for p, _ in
                                                                                              self.params}:
            optimizer._param_groups = []
            optimizer._add_param_group({"params": [p for p, _ in self.params]})
            optimizer._parameter_list = [p for p, _ in self.params]
        # producer stage of every variable, and the stages reading it
        self.producer_stage = {}
        for op in self.fwd_ops + self.bwd_ops:
            for v in P._iter_vars(op.outputs):
                self.producer_stage[id(v)] = self.op_stage[id(op)]
        self.consumers = {}
        for op in self.fwd_ops + self.bwd_ops:
            st = self.op_stage[id(op)]
            for v in self._inputs(op):
                ps = self.producer_stage.get(id(v))
                if ps is not None and ps != st:
                    self.consumers.setdefault(id(v), set()).add(st)
        # Message order. RCCL pairs point-to-point messages by posting order, not by tag, so the
        # receiver must post its receives in exactly the order the sender posts its sends. Each
        # (src -> dst) stream is laid out statically: every section in run order (forward of micro-
        # batches 0..k-1, then their backward), the producer stage's ops in program order, each
        # op's outputs that dst reads. A receive that needs the n-th message of a stream first
        # takes messages 0..n-1 (buffered into their micro-batch's environment) — always safe, as
        # the sender posted them before the n-th.
        self.streams = {}
        sections = [(self.fwd_ops, m) for m in range(self.k)] + [(self.bwd_ops, m) for m in range(self.k)]
        for ops, m in sections:
            for op in ops:
                src = self.op_stage[id(op)]
                for v in P._iter_vars(op.outputs):
                    for dst in sorted(self.consumers.get(id(v), ())):
                        if dst != src:
                            self.streams.setdefault((src, dst), []).append((m, id(v)))

    def _inputs(self, op):
        return [v for v in B._op_inputs(self.prog, op) if isinstance(v, P.Variable)]

    def _recv_until(self, src, m, vid, envs, xfer):
        seq = self.streams.get((src, self.stage), [])
        cur = self._cursor.get(src, 0)
        while vid not in envs[m]:
            if cur >= len(seq):
                raise RuntimeError(f"static pipeline: stage {self.stage} needs a variable stage {src} never sends")
            mm, want = seq[cur]
            t = xfer.recv(src, cur, self.device)
            if t.is_floating_point():
                t.requires_grad_(True)
            envs[mm][want] = _wrap(t)
            cur += 1
        self._cursor[src] = cur

    def _section(self, ops, envs, m, xfer):
        """run this stage's ops of ``ops`` for micro-batch m, with the transfers around them"""
        me = self.stage
        env = envs[m]
        fake = P.Block(self.prog)
        for op in ops:
            st = self.op_stage[id(op)]
            if st == me:
                for v in self._inputs(op):
                    ps = self.producer_stage.get(id(v))
                    if ps is not None and ps != me and id(v) not in env:
                        self._recv_until(ps, m, id(v), envs, xfer)
                fake.ops = [op]
                P.run_block(self.prog, fake, env)
                for v in P._iter_vars(op.outputs):
                    for cs in sorted(self.consumers.get(id(v), ())):
                        if cs != me:
                            if id(v) not in env:
                                raise RuntimeError(f"static pipeline: {v.name} was not produced on stage {me}")
                            n = self._sent.get(cs, 0)
                            xfer.send(env[id(v)]._t, cs, n)
                            self._sent[cs] = n + 1

    @property
    def device(self):
        from ...framework import core as _c
        return _c.default_device()

    def run(self, feed, fetch_list):
        blk = self.prog.global_block()
        parts = {}
        for name, val in feed.items():
            a = val.numpy() if isinstance(val, Tensor) else np.asarray(val)
            parts[name] = np.array_split(a, self.k, axis=0)
        xfer = _Transfer(self)
        self._cursor, self._sent = {}, {}
        envs = []
        for m in range(self.k):
            env = {}
            for name, chunks in parts.items():
                v = blk.vars.get(name)
                if v is None:
                    continue
                t = torch.as_tensor(chunks[m], device=self.device)
                if t.dtype != v._t.dtype:
                    t = t.to(v._t.dtype)
                if getattr(v, "need_grad", False) and t.is_floating_point():
                    t.requires_grad_(True)
                env[id(v)] = _wrap(t)
            envs.append(env)
        for m in range(self.k):
            self._section(self.fwd_ops, envs, m, xfer)
        for m in range(self.k):
            self._section(self.bwd_ops, envs, m, xfer)
        xfer.wait()
        # average the parameter gradients over the micro-batches, then the inner optimizer
        with torch.no_grad():
            for p, g in self.params:
                acc = None
                for env in envs:
                    gv = env.get(id(g))
                    if gv is None:
                        continue
                    acc = gv._t.detach().float() if acc is None else acc + gv._t.detach().float()
                if acc is not None:
                    p._t.grad = (acc / self.k).to(p._t.dtype)
        with P._core_dynamic():
            if self.params:
                self.opt.step()
                self.opt.clear_grad(set_to_zero=False)
        res = []
        for f in fetch_list:
            v = blk.vars[f] if isinstance(f, str) else f
            vals = [env[id(v)]._t.detach() for env in envs if id(v) in env]
            if not vals:
                res.append(None)
            elif vals[0].dim() == 0 or vals[0].numel() == 1:
                res.append(_wrap(torch.stack([x.float().reshape(()) for x in vals]).mean().reshape(vals[0].shape)))
            else:
                res.append(_wrap(torch.cat(vals, 0)))
        return res


class PipelineOptimizer:
    """``fleet.distributed_optimizer(opt, strategy)`` with ``strategy.pipeline = True`` (and
    ``fluid.optimizer.PipelineOptimizer``) in static mode: per-op backward, then the program is
    marked for the pipeline runner of this rank's stage."""

    def __init__(self, inner, num_microbatches=1, n_stages=None, stage=None, ranks=None, group=None):
        self.inner = inner
        self.k = num_microbatches
        world = tdist.get_world_size() if tdist.is_initialized() else 1
        self.n_stages = n_stages or world
        self.stage = stage if stage is not None else (tdist.get_rank() if tdist.is_initialized() else 0)
        self.ranks, self.group = ranks, group

    def __getattr__(self, item):
        return getattr(self.inner, item)

    def minimize(self, loss, startup_program=None, parameter_list=None, no_grad_set=None):
        prog = P.default_main_program()
        params = parameter_list if parameter_list is not None else [p for p in prog.all_parameters() if p.trainable]
        pg = B.append_backward(loss, params, no_grad_set)
        prog.__dict__["_pipeline"] = PipelineRunner(prog, self.inner, pg, self.n_stages, self.stage, self.k,
                                                    self.ranks, self.group)
        return [], pg
