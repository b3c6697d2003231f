"""Planner: choose the sharding of the weights when the user annotates none (or some).

Reference: python/paddle/distributed/auto_parallel/planner_v2.py:22 (Planner over the cost model:
search the distributed attributes of ops / tensors that minimise the estimated step time).

Search space: every 2-D weight (``linear`` weight, ``matmul`` operand that is a parameter) is
replicated, column-split or row-split along one mesh dim. A candidate plan is priced by running
completion on it and summing, per op, MFMA time of the local GEMM share plus ring-collective
time over xGMI of every communication completion implies (partial-sum all-reduces, all-gathers of
inputs whose split a consumer cannot take, and the backward all-reduce of inputs replicated
across a split computation), with a penalty above the per-rank parameter memory budget.
Coordinate descent from all-replicated, two sweeps. A col -> row Megatron pair (one all-reduce
per pair) is what this search lands on for MLP / attention blocks under memory pressure.
"""
from __future__ import annotations

import numpy as np

from ...framework.core import Parameter, Tensor
from ...static.program import Variable
from .completion import Completer, _short, dims_of
from .cost_model import MI355X, _ring


def _weights(program):
    out, seen = [], set()
    for op in program.global_block().ops:
        name = _short(op.type)
        w = op.kwargs.get("weight") if name == "linear" else op.kwargs.get("y") if name == "matmul" else None
        if isinstance(w, Parameter) and w._t.dim() == 2 and id(w) not in seen:
            seen.add(id(w))
            out.append(w)
    return out


def _bytes(t):
    return int(np.prod(dims_of(t))) * t._t.element_size()


def plan_cost(program, mesh, hw=None, memory_limit=None):
    hw = dict(MI355X, **(hw or {}))
    comp = Completer(mesh).complete(program)
    topo = mesh.topology
    bw = hw["xgmi_link_bw"] * hw["xgmi_links"] / 2
    lat = hw["collective_latency"]
    t_compute = t_comm = 0.0
    for op in program.global_block().ops:
        d = comp.ops.get(id(op))
        if d is None:
            continue
        name = _short(op.type)
        split = {m for m in (d.output or []) if m >= 0} | set(d.partial)
        shards = int(np.prod([topo[m] for m in split])) if split else 1
        if name in ("linear", "matmul"):
            x = op.kwargs["x"]
            w = op.kwargs.get("weight", op.kwargs.get("y"))
            xs, ws = dims_of(x), dims_of(w)
            flops = 2.0 * np.prod(xs) * ws[-1]
            t_compute += flops / shards / (hw["bf16_flops"] * hw["mfma_efficiency"])
        out = op.outputs
        if d.partial and isinstance(out, Variable):
            for m in d.partial:
                t_comm += _ring(_bytes(out), topo[m], bw, lat)
        for k, v in op.kwargs.items():
            req = d.inputs.get(k)
            if not isinstance(v, Variable) or req is None:
                continue
            cur = comp.dm.get(id(v), [-1] * len(req))
            for c, r in zip(cur, req):
                if c >= 0 and c != r:      # all-gather (half a ring all-reduce)
                    t_comm += _ring(_bytes(v), topo[c], bw, lat) / 2
            for m in split - {x for x in req if x >= 0}:
                if v._t.is_floating_point():
                    t_comm += _ring(_bytes(v), topo[m], bw, lat)   # backward all-reduce of its gradient
    mem = 0.0
    for t in {id(t): t for t in _params(program)}.values():
        dm = comp.dm.get(id(t)) or [-1] * t._t.dim()
        mem += _bytes(t) / int(np.prod([topo[m] for m in dm if m >= 0] or [1]))
    # parameter + gradient + 2 Adam moments (fp32) per byte of bf16 weight: x8
    penalty = 0.0 if memory_limit is None or mem * 8 <= memory_limit else 1e3 * (mem * 8 / memory_limit)
    return {"compute": t_compute, "comm": t_comm, "param_bytes": mem, "total": t_compute + t_comm + penalty}


def _params(program):
    for op in program.global_block().ops:
        for v in op.kwargs.values():
            if isinstance(v, Parameter):
                yield v


def plan(program, mesh, mesh_dim=0, memory_limit=None, hw=None, sweeps=2):
    """annotate the unannotated 2-D weights of ``program`` (``dist_attr``) with the cheapest
    replicate / column / row choice; -> (assignment {weight name: dims_mapping}, cost dict)"""
    m = mesh.dim_index(mesh_dim)
    ws = [w for w in _weights(program) if (getattr(w, "dist_attr", None) or {}).get("dims_mapping") is None]
    options = [[-1, -1], [-1, m], [m, -1]]
    choice = {id(w): 0 for w in ws}

    def apply():
        for w in ws:
            w.dist_attr = {"process_mesh": mesh, "dims_mapping": list(options[choice[id(w)]])}

    def clear():
        for w in ws:
            w.dist_attr = None

    apply()
    best = plan_cost(program, mesh, hw, memory_limit)
    for _ in range(sweeps):
        improved = False
        for w in ws:
            keep = choice[id(w)]
            for o in range(len(options)):
                if o == keep:
                    continue
                choice[id(w)] = o
                apply()
                c = plan_cost(program, mesh, hw, memory_limit)
                if c["total"] < best["total"] * (1 - 1e-9):
                    best, keep, improved = c, o, True
            choice[id(w)] = keep
            apply()
        if not improved:
            break
    return {w.name: list(options[choice[id(w)]]) for w in ws}, best
