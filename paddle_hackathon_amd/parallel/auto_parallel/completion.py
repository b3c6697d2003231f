"""Completion: propagate ``dims_mapping`` annotations through a static Program.

Reference: python/paddle/distributed/auto_parallel/completion.py:140 (Completer.complete_forward_
annotation: per-op SPMD rules from operators/dist_*.py decide the distributed attributes of every
unannotated tensor and op). A dims_mapping lists, per tensor dim, the mesh dim it is split along
(-1 = replicated).

``complete(program, mesh)`` walks the ops of block 0 in order. Each op's rule sees the current
mappings of its tensor inputs (None = unannotated parameter / constant, free to choose) and
returns the mappings it needs for its inputs, the mapping of its output and the mesh dims along
which the output is a partial sum (``partial``, resolved by an all-reduce right after the op).
Unannotated parameters take the mapping the rule asks for — that is how annotating one weight of
a Megatron pair determines the other (x[.., k] split on m => W[k, n] row-split on m => output
partial on m). Ops without a rule run replicated.
"""
from __future__ import annotations

from ...framework.core import Tensor
from ...static import program as P
from ...static.program import Variable, _iter_vars

_PKG = "paddle_hackathon_amd."


def _short(op_type):
    return op_type.rsplit(".", 1)[-1]


def dims_of(t):
    """logical (global) shape of a tensor / Variable (declared batch dims -> meta size)"""
    return list(t._t.shape)


def annotation(t):
    da = getattr(t, "dist_attr", None)
    if isinstance(da, dict) and da.get("dims_mapping") is not None:
        return list(da["dims_mapping"])
    return None


class OpDist:
    """completion result of one op"""
    __slots__ = ("inputs", "output", "partial", "reduce", "rule")

    def __init__(self, inputs, output, partial=(), reduce="sum", rule="replicated"):
        self.inputs = inputs            # {kwarg name: required dims_mapping} for tensor kwargs
        self.output = output            # dims_mapping of the (single) output, or None
        self.partial = tuple(partial)   # mesh dims the output is a partial sum / mean over
        self.reduce = reduce            # "sum" | "avg"
        self.rule = rule

    def __repr__(self):
        return f"OpDist({self.rule}: in={self.inputs} out={self.output} partial={self.partial})"


def _merge_elementwise(dms, shapes, out_ndim):
    out = [-1] * out_ndim
    for dm, shp in zip(dms, shapes):
        if dm is None:
            continue
        off = out_ndim - len(dm)
        for i, m in enumerate(dm):
            if m >= 0 and shp[i] != 1 and out[off + i] == -1 and m not in out:
                out[off + i] = m
    return out


def _align(dm_out, shp):
    """the mapping an input of shape ``shp`` needs to match an elementwise output mapping"""
    off = len(dm_out) - len(shp)
    return [(-1 if shp[i] == 1 else dm_out[off + i]) for i in range(len(shp))]


ELEMENTWISE = {"add", "subtract", "multiply", "divide", "maximum", "minimum", "pow", "relu", "gelu", "tanh",
               "sigmoid", "silu", "swish", "exp", "sqrt", "rsqrt", "scale", "dropout", "cast", "abs", "neg",
               "square", "log", "erf", "leaky_relu", "elu", "relu6", "hardswish", "mish", "softplus", "clip", "where",
               "bias_gelu", "fused_dropout_add"}
NORMS_LAST = {"softmax", "log_softmax", "layer_norm"}
REDUCES = {"sum", "mean"}


class Completer:
    def __init__(self, mesh):
        self.mesh = mesh
        self.dm = {}          # id(tensor) -> dims_mapping
        self.ops = {}         # id(op) -> OpDist

    # -------------------------------------------------------------------------- helpers
    def get(self, t):
        if id(t) in self.dm:
            return self.dm[id(t)]
        a = annotation(t)
        if a is not None:
            self.dm[id(t)] = a
            return a
        if isinstance(t, Variable):
            # unannotated data / intermediate: replicated
            self.dm[id(t)] = [-1] * len(dims_of(t))
            return self.dm[id(t)]
        return None           # unannotated parameter / constant: the rule chooses

    def set(self, t, dm):
        if isinstance(t, Tensor) and id(t) not in self.dm:
            self.dm[id(t)] = list(dm)

    def complete(self, program):
        for op in program.global_block().ops:
            if P.is_train_op(op) or op.exec is not None:
                continue
            d = self.rule(op)
            self.ops[id(op)] = d
            for k, dm in d.inputs.items():
                v = op.kwargs.get(k)
                if isinstance(v, Tensor) and id(v) not in self.dm and dm is not None:
                    self.dm[id(v)] = list(dm)
            out = op.outputs
            if isinstance(out, Variable) and d.output is not None:
                self.dm[id(out)] = list(d.output)
            elif isinstance(out, (list, tuple)):
                for v in _iter_vars(out):
                    self.dm.setdefault(id(v), [-1] * len(dims_of(v)))
        return self

    # -------------------------------------------------------------------------- rules
    def rule(self, op):
        name = _short(op.type)
        kw = op.kwargs
        fn = getattr(self, f"_rule_{name}", None)
        if fn is not None:
            return fn(kw)
        if name in ELEMENTWISE:
            return self._elementwise(kw)
        if name in NORMS_LAST:
            return self._norm_last(kw, name)
        if name in REDUCES:
            return self._reduce(kw, name)
        return self._replicated(op)

    def _tensor_kwargs(self, kw):
        return {k: v for k, v in kw.items() if isinstance(v, Tensor)}

    def _replicated(self, op):
        ins = {k: [-1] * len(dims_of(v)) for k, v in self._tensor_kwargs(op.kwargs).items()}
        out = op.outputs
        od = [-1] * len(dims_of(out)) if isinstance(out, Variable) else None
        return OpDist(ins, od, rule="replicated")

    def _elementwise(self, kw):
        ts = self._tensor_kwargs(kw)
        shapes = {k: dims_of(v) for k, v in ts.items()}
        nd = max((len(s) for s in shapes.values()), default=0)
        out = _merge_elementwise([self.get(v) for v in ts.values()], list(shapes.values()), nd)
        ins = {k: _align(out, shapes[k]) for k in ts}
        return OpDist(ins, out, rule="elementwise")

    def _norm_last(self, kw, name):
        x = kw["x"]
        dm = list(self.get(x))
        shp = dims_of(x)
        if name == "layer_norm":
            ns = kw.get("normalized_shape")
            nn_ = 1 if isinstance(ns, int) else len(ns)
            for i in range(len(dm) - nn_, len(dm)):
                dm[i] = -1
            ins = {"x": dm}
            for k in ("weight", "bias"):
                if isinstance(kw.get(k), Tensor):
                    ins[k] = [-1] * len(dims_of(kw[k]))
            return OpDist(ins, dm, rule="norm")
        axis = kw.get("axis", -1)
        axis = axis % len(shp)
        dm[axis] = -1
        return OpDist({"x": dm}, dm, rule="norm")

    def _reduce(self, kw, name):
        x = kw["x"]
        dm = self.get(x)
        nd = len(dm)
        axis = kw.get("axis")
        axes = list(range(nd)) if axis is None else ([axis] if isinstance(axis, int) else list(axis))
        axes = [a % nd for a in axes] if nd else []
        keep = kw.get("keepdim", False)
        partial = tuple(sorted({dm[a] for a in axes if dm[a] >= 0}))
        out = [(-1 if i in axes else m) for i, m in enumerate(dm)] if keep else [m for i, m in enumerate(dm) if i not in axes]
        if not out and nd:
            out = []
        return OpDist({"x": dm}, out, partial, "avg" if name == "mean" else "sum", rule="reduce")

    def _rule_transpose(self, kw):
        dm = self.get(kw["x"])
        return OpDist({"x": dm}, [dm[p] for p in kw["perm"]], rule="transpose")

    def _rule_reshape(self, kw):
        x = kw["x"]
        dm = self.get(x)
        ish = dims_of(x)
        osh = _resolve_shape(ish, kw["shape"])
        out = [-1] * len(osh)
        need = list(dm)
        for i, m in enumerate(dm):
            if m < 0:
                continue
            pre = _prod(ish[:i])
            j = next((j for j in range(len(osh)) if _prod(osh[:j]) == pre), None)
            n = self.mesh.topology[m]
            if j is not None and osh[j] % n == 0 and (ish[i] == osh[j] or (ish[i] % osh[j] == 0) or
                                                      (osh[j] % n == 0 and _prod(osh[j:]) == _prod(ish[i:]))):
                out[j] = m
            else:
                need[i] = -1          # split dim does not survive: gather it first
        return OpDist({"x": need}, out, rule="reshape")

    def _matmul_like(self, x, y, tx, ty, has_bias=False, bias=None):
        xs, ys = dims_of(x), dims_of(y)
        dx = list(self.get(x))
        dy = self.get(y)
        xk = len(xs) - (2 if tx else 1)            # index of the contracting dim of x
        if len(ys) == 1:
            yk, yn = 0, None
        else:
            yk, yn = (len(ys) - 1, len(ys) - 2) if ty else (len(ys) - 2, len(ys) - 1)
        if dy is None:                              # unannotated weight: follow x's k split
            dy = [-1] * len(ys)
            dy[yk] = dx[xk]
        dy = list(dy)
        k = dx[xk] if dx[xk] >= 0 else dy[yk]
        if dx[xk] >= 0 and dy[yk] >= 0 and dx[xk] != dy[yk]:
            k = dx[xk]
        dx[xk] = k
        dy[yk] = k
        n_m = dy[yn] if yn is not None else -1
        if n_m >= 0 and n_m in dx:
            n_m = -1
            dy[yn] = -1
        # output: x's batch / row dims + n
        if len(xs) >= 2:
            xm = len(xs) - (1 if tx else 2)
            out = [dx[i] for i in range(len(xs) - 2)] + [dx[xm]]
        else:
            out = []
        if yn is not None:
            out = out + [n_m]
        # y's batch dims (attention: [B, H, S, D]) follow x's
        if len(ys) > 2 and len(xs) == len(ys):
            for i in range(len(ys) - 2):
                dy[i] = dx[i]
        ins = {"x": dx, "y": dy}
        partial = (k,) if k >= 0 else ()
        return ins, out, partial

    def _rule_matmul(self, kw):
        ins, out, partial = self._matmul_like(kw["x"], kw["y"], kw.get("transpose_x", False),
                                              kw.get("transpose_y", False))
        return OpDist(ins, out, partial, rule="matmul")

    def _rule_linear(self, kw):
        ins, out, partial = self._matmul_like(kw["x"], kw["weight"], False, False)
        d = {"x": ins["x"], "weight": ins["y"]}
        if isinstance(kw.get("bias"), Tensor):
            d["bias"] = [ins["y"][1]]
        return OpDist(d, out, partial, rule="linear")

    def _rule_embedding(self, kw):
        x, w = kw["x"], kw["weight"]
        dx = self.get(x)
        dw = self.get(w)
        h = -1 if dw is None else dw[1]
        if h in dx:
            h = -1
        return OpDist({"x": dx, "weight": [-1, h]}, list(dx) + [h], rule="embedding")

    def _rule_cross_entropy(self, kw):
        x, lab = kw["input"], kw["label"]
        dx = list(self.get(x))
        dx[-1] = -1
        red = kw.get("reduction", "mean")
        batch = dx[:-1]
        dl = self.get(lab)
        dl = list(batch) + ([-1] if len(dims_of(lab)) == len(dims_of(x)) else [])
        if red == "none":
            return OpDist({"input": dx, "label": dl}, batch + [-1], rule="cross_entropy")
        partial = tuple(sorted({m for m in batch if m >= 0}))
        return OpDist({"input": dx, "label": dl}, [], partial, "avg" if red == "mean" else "sum", rule="cross_entropy")

    def _rule_mse_loss(self, kw):
        x, y = kw["input"], kw["label"]
        dx = list(self.get(x))
        red = kw.get("reduction", "mean")
        ins = {"input": dx, "label": _align(dx, dims_of(y))}
        if red == "none":
            return OpDist(ins, dx, rule="mse_loss")
        partial = tuple(sorted({m for m in dx if m >= 0}))
        return OpDist(ins, [], partial, "avg" if red == "mean" else "sum", rule="mse_loss")


def _prod(xs):
    p = 1
    for v in xs:
        p *= int(v)
    return p


def _resolve_shape(ish, shape):
    shape = [int(s) if not isinstance(s, Tensor) else int(s._t.reshape(-1)[0]) for s in shape]
    out = [ish[i] if s == 0 else s for i, s in enumerate(shape)]
    if -1 in out:
        known = _prod([s for s in out if s != -1])
        out[out.index(-1)] = _prod(ish) // max(1, known)
    return out


def complete(program, mesh):
    return Completer(mesh).complete(program)
