"""Static-graph quantization passes (reference: python/paddle/fluid/contrib/slim/quantization/
quantization_pass.py:35-47 — QuantizationTransformPass, QuantizationFreezePass, ConvertToInt8Pass,
TransformForMobilePass, OutScaleForTrainingPass, OutScaleForInferencePass, AddQuantDequantPass,
QuantizationTransformPassV2, AddQuantDequantPassV2, ReplaceFakeQuantDequantPass, QuantWeightPass).

The reference rewrites an ``IrGraph`` (core.Graph over the ProgramDesc). Here a pass rewrites the
Program's op list directly (``IrGraph`` is a thin view over a Program, so reference scripts that
build ``IrGraph(core.Graph(program.desc))`` and call ``graph.to_program()`` work unchanged).
Quantizable ops and their activation / weight operands are found by reference op type and slot
(static/serialize.py op_reference), so programs recorded through the paddle API and programs
loaded from reference ProgramDescs are handled alike. The inserted ops are the fake-quant ops of
nn/quant/ops.py (HIP kernels on the GPU; written back as the reference op types)."""
from __future__ import annotations

import numpy as np
import torch

from .....framework.core import Parameter, Tensor, _wrap
from .....static import program as P
from .....static.serialize import op_reference

__all__ = ["QuantizationTransformPass", "QuantizationFreezePass", "ConvertToInt8Pass", "TransformForMobilePass",
           "OutScaleForTrainingPass", "OutScaleForInferencePass", "AddQuantDequantPass", "QuantizationTransformPassV2",
           "AddQuantDequantPassV2", "ReplaceFakeQuantDequantPass", "QuantWeightPass", "IrGraph"]

# reference op type -> (activation slot, weight slot, weight channel axis)
QUANT_OPS = {"conv2d": ("Input", "Filter", 0), "depthwise_conv2d": ("Input", "Filter", 0),
             "conv2d_transpose": ("Input", "Filter", 1), "mul": ("X", "Y", 1), "matmul": ("X", "Y", 1),
             "matmul_v2": ("X", "Y", 1), "fc": ("Input", "W", 1)}
# ops whose float inputs AddQuantDequantPass quantizes (reference _op_real_in_out_name subset)
QDQ_OPS = ("elementwise_add", "elementwise_sub", "elementwise_mul", "pool2d", "concat", "relu", "relu6",
           "leaky_relu", "sigmoid", "tanh", "hard_swish", "swish", "reshape2", "transpose2", "flatten2",
           "flatten_contiguous_range", "bmm", "matmul_v2", "batch_norm", "layer_norm", "softmax", "scale")
_FAKE_QDQ = ("fake_quantize_dequantize_abs_max", "fake_quantize_dequantize_moving_average_abs_max",
             "fake_channel_wise_quantize_dequantize_abs_max")


def _qo():
    from .....nn.quant import ops as QO
    return QO


class IrGraph:
    """``fluid.framework.IrGraph`` stand-in: a view over a Program (``core.Graph(program.desc)``
    yields the Program itself)"""

    def __init__(self, graph, for_test=False):
        self.program = graph.program if isinstance(graph, IrGraph) else graph
        self._for_test = for_test

    def to_program(self):
        return self.program

    def is_test(self):
        return self._for_test

    def clone(self):
        return IrGraph(self.program.clone(), self._for_test)

    def all_op_nodes(self):
        return list(self.program.global_block().ops)

    def all_var_nodes(self):
        return list(self.program.global_block().vars.values())

    def draw(self, save_path, name, marked_nodes=None, remove_ctr_var=True):
        return None


def _prog(graph):
    return graph.program if isinstance(graph, IrGraph) else graph


def _ret(graph, prog):
    return graph if isinstance(graph, IrGraph) else prog


def _state(value, shape=(1,), name="quant_state"):
    """a persistable fp32 state tensor (scale / moving-average state), saved with the program"""
    from .....framework import core as _core
    dev = _core.default_device()
    p = Parameter(data=torch.full(shape, float(value), dtype=torch.float32, device=dev), name=_unique(name),
                  trainable=False)
    p.stop_gradient = True
    return p


def _unique(prefix):
    from .....utils import unique_name
    return unique_name.generate(prefix)


def _new_var(blk, like, name):
    meta = like._t if like._t.device.type == "meta" else like._t.to("meta")
    v = P.Variable(blk, meta, _unique(name))
    blk.vars[v.name] = v
    return v


def _replace_input(op, kwarg, new):
    old = op.kwargs[kwarg]
    op.kwargs = dict(op.kwargs)
    op.kwargs[kwarg] = new
    r = op.attrs.get("ref_op")
    if r is not None:
        for ts in r[1].values():
            for i, t in enumerate(ts):
                if t is old:
                    ts[i] = new


def _insert_before(blk, op, new_op):
    blk.ops.insert(blk.ops.index(op), new_op)
    for v in P._iter_vars(new_op.outputs):
        v.op = new_op


def _make_op(fn_name, kwargs, out, attrs=None):
    QO = _qo()
    fn = getattr(QO, fn_name)
    fn = getattr(fn, "__wrapped_op__", fn)
    return P.OpDesc(f"{fn.__module__}.{fn.__name__}", fn, (), kwargs, out, attrs or {})


def _skipped(op, skip_pattern):
    scope = op.attrs.get("name_scope", "") or ""
    return bool(op.attrs.get("skip_quant")) or any(p and p in scope for p in (skip_pattern or []))


def _quantizable(prog, types, skip_pattern=()):
    """-> [(op, activation kwarg, weight kwarg | None, weight axis)] in program order"""
    out = []
    for op in list(prog.global_block().ops):
        ref = op_reference(op)
        if ref is None or ref[0] not in types or _skipped(op, skip_pattern) or P.is_train_op(op):
            continue
        typ, slots = ref
        a_slot, w_slot, axis = QUANT_OPS.get(typ, ("X", None, 0))
        act = slots.get(a_slot)
        w = slots.get(w_slot) if w_slot else None
        if act is None:
            continue
        wt = op.kwargs.get(w) if w else None
        out.append((op, act, w if isinstance(wt, Tensor) else None, axis))
    return out


def _is_weight(t):
    return isinstance(t, Tensor) and not isinstance(t, P.Variable)


# ------------------------------------------------------------------------------------- transform
class QuantizationTransformPass:
    """insert fake quant-dequant ops on the activation and weight inputs of the quantizable ops
    of a TRAINING program (apply before append_backward / minimize; the ops carry straight-through
    gradients). activation_quantize_type: 'abs_max' | 'moving_average_abs_max' | 'range_abs_max'
    (= moving average here); weight_quantize_type: 'abs_max' | 'channel_wise_abs_max'."""

    def __init__(self, scope=None, place=None, weight_bits=8, activation_bits=8, activation_quantize_type="abs_max",
                 weight_quantize_type="abs_max", window_size=10000, moving_rate=0.9, skip_pattern=("skip_quant",),
                 quantizable_op_type=("conv2d", "depthwise_conv2d", "mul"), weight_quantize_func=None,
                 act_quantize_func=None, weight_preprocess_func=None, act_preprocess_func=None,
                 optimizer_func=None, executor=None, is_test=None):
        if activation_quantize_type not in ("abs_max", "moving_average_abs_max", "range_abs_max"):
            raise ValueError(f"Unknown activation_quantize_type {activation_quantize_type!r}")
        if weight_quantize_type not in ("abs_max", "channel_wise_abs_max"):
            raise ValueError(f"Unknown weight_quantize_type {weight_quantize_type!r}")
        self._wbits, self._abits = weight_bits, activation_bits
        self._atype, self._wtype = activation_quantize_type, weight_quantize_type
        self._rate = moving_rate
        self._skip = list(skip_pattern) if isinstance(skip_pattern, (list, tuple)) else [skip_pattern]
        self._types = tuple(quantizable_op_type)
        self._is_test = is_test
        self._cache = {}

    def _act_quant(self, blk, v):
        if id(v) in self._cache:
            return self._cache[id(v)]
        out = _new_var(blk, v, (getattr(v, "name", "x") or "x") + ".quantized.dequantized")
        if self._atype == "abs_max":
            sv = _new_var(blk, _wrap(torch.empty(1, device="meta")), "quant.scale")
            op = _make_op("fake_quantize_dequantize_abs_max", {"x": v, "bit_length": self._abits}, (out, sv))
        else:
            op = _make_op("fake_quantize_dequantize_moving_average_abs_max",
                          {"x": v, "in_scale": _state(0.001, name="quant.scale"),
                           "in_state": _state(1.0, name="quant.state"), "in_accum": _state(1.0, name="quant.accum"),
                           "bit_length": self._abits, "moving_rate": self._rate, "is_test": bool(self._is_test)}, out)
        self._cache[id(v)] = (out, op)
        return out, op

    def _weight_quant(self, blk, w, axis):
        if id(w) in self._cache:
            return self._cache[id(w)]
        like = _wrap(w._t.to("meta"))
        out = _new_var(blk, like, (getattr(w, "name", "w") or "w") + ".quantized.dequantized")
        sv = _new_var(blk, _wrap(torch.empty(w._t.shape[axis] if self._wtype != "abs_max" else 1, device="meta")),
                      "quant.scale")
        if self._wtype == "abs_max":
            op = _make_op("fake_quantize_dequantize_abs_max", {"x": w, "bit_length": self._wbits}, (out, sv))
        else:
            op = _make_op("fake_channel_wise_quantize_dequantize_abs_max",
                          {"x": w, "bit_length": self._wbits, "quant_axis": axis}, (out, sv))
        op.attrs["quantized_weight"] = True
        self._cache[id(w)] = (out, op)
        return out, op

    def apply(self, graph):
        prog = _prog(graph)
        blk = prog.global_block()
        for op, act, w, axis in _quantizable(prog, self._types, self._skip):
            v = op.kwargs[act]
            if isinstance(v, Tensor) and v._t.is_floating_point():
                q, qop = self._act_quant(blk, v)
                if qop not in blk.ops:
                    _insert_before(blk, op, qop)
                _replace_input(op, act, q)
            if w is not None and _is_weight(op.kwargs[w]):
                q, qop = self._weight_quant(blk, op.kwargs[w], axis)
                if qop not in blk.ops:
                    _insert_before(blk, op, qop)
                _replace_input(op, w, q)
            op.attrs.setdefault("extra_attrs", {})["with_quant_attr"] = True
        return _ret(graph, prog)


class AddQuantDequantPass:
    """moving-average fake quant-dequant on the float inputs of ``quantizable_op_type`` ops
    (element-wise / pooling / activation ops) that QuantizationTransformPass does not cover"""

    def __init__(self, scope=None, place=None, moving_rate=0.9, quant_bits=8, skip_pattern=("skip_quant",),
                 quantizable_op_type=("elementwise_add", "pool2d"), is_full_quantized=False, is_test=None):
        self._bits, self._rate = quant_bits, moving_rate
        self._skip = list(skip_pattern) if isinstance(skip_pattern, (list, tuple)) else [skip_pattern]
        self._types = QDQ_OPS if is_full_quantized else tuple(quantizable_op_type)
        self._is_test = is_test

    def apply(self, graph):
        prog = _prog(graph)
        blk = prog.global_block()
        cache = {}
        for op in list(blk.ops):
            ref = op_reference(op)
            if ref is None or ref[0] not in self._types or _skipped(op, self._skip) or P.is_train_op(op):
                continue
            for slot, k in ref[1].items():
                v = op.kwargs.get(k)
                if not isinstance(v, P.Variable) or not v._t.is_floating_point():
                    continue
                if id(v) not in cache:
                    out = _new_var(blk, v, (v.name or "x") + ".quant_dequant")
                    q = _make_op("fake_quantize_dequantize_moving_average_abs_max",
                                 {"x": v, "in_scale": _state(0.001, name="quant_dequant.scale"),
                                  "in_state": _state(1.0, name="quant_dequant.state"),
                                  "in_accum": _state(1.0, name="quant_dequant.accum"), "bit_length": self._bits,
                                  "moving_rate": self._rate, "is_test": bool(self._is_test)}, out)
                    _insert_before(blk, op, q)
                    cache[id(v)] = out
                _replace_input(op, k, cache[id(v)])
        return _ret(graph, prog)


# ---------------------------------------------------------------------------------------- freeze
def _qdq_value(w, scale, bits, axis=None):
    from .....ops import quant as Q
    return Q.quant_dequant(w, scale, bits, 1, quant_axis=axis)


def _ref_type(op):
    r = op_reference(op)
    return r[0] if r else None


class QuantizationFreezePass:
    """an inference program from a quantization-trained one: weights are quantized once into their
    parameters (the fake-quant weight ops removed), the activation fake-quant ops keep their
    trained scales and run as frozen (is_test) quant-dequant"""

    def __init__(self, scope=None, place=None, bias_correction=False, weight_bits=8, activation_bits=8,
                 weight_quantize_type="abs_max", quantizable_op_type=None, round_type="round"):
        self._wbits, self._abits = weight_bits, activation_bits

    def apply(self, graph):
        prog = _prog(graph)
        blk = prog.global_block()
        rewire = {}
        keep = []
        for op in blk.ops:
            typ = _ref_type(op)
            w = op.kwargs.get("x")
            if typ in ("fake_quantize_dequantize_abs_max", "fake_channel_wise_quantize_dequantize_abs_max") \
                    and _is_weight(w):
                from .....ops import quant as Q
                axis = op.kwargs.get("quant_axis") if typ.startswith("fake_channel") else None
                s = Q.channel_abs_max(w._t, axis) if axis is not None else Q.abs_max(w._t)
                with torch.no_grad():
                    w._t.copy_(_qdq_value(w._t, s, op.kwargs.get("bit_length", self._wbits), axis).to(w._t.dtype))
                w._frozen_quant = (s.detach().clone(), axis)   # ConvertToInt8Pass stores on this grid
                outs = op.outputs if isinstance(op.outputs, (tuple, list)) else (op.outputs,)
                rewire[id(outs[0])] = w
                continue
            if typ in ("fake_quantize_dequantize_moving_average_abs_max", "moving_average_abs_max_scale"):
                op.kwargs = dict(op.kwargs, is_test=True)
            keep.append(op)
        for op in keep:
            for k, v in list(op.kwargs.items()):
                if id(v) in rewire:
                    _replace_input(op, k, rewire[id(v)])
        blk.ops = keep
        return _ret(graph, prog)


class ConvertToInt8Pass:
    """stores each frozen weight as int8 levels plus its per-channel scale; a dequantize_linear op
    rebuilds the float weight in the program (8-bit weights on disk and in HBM)"""

    def __init__(self, scope=None, place=None, quantizable_op_type=None, weight_bits=8):
        self._bits = weight_bits
        self._types = tuple(quantizable_op_type or QUANT_OPS)

    def apply(self, graph):
        prog = _prog(graph)
        blk = prog.global_block()
        done = {}
        from .....ops import quant as Q
        for op, act, w, axis in _quantizable(prog, self._types):
            if w is None:
                continue
            wt = op.kwargs[w]
            if not isinstance(wt, Parameter):
                continue
            if id(wt) not in done:
                frozen = getattr(wt, "_frozen_quant", None)
                if frozen is not None:   # the freeze pass's own scale (per tensor or per channel)
                    s, qaxis = frozen
                else:
                    s, qaxis = Q.channel_abs_max(wt._t, axis), axis
                if qaxis is None:
                    s = s.reshape(-1)[:1].float()
                lv = Q.quant_dequant(wt._t, s, self._bits, 0, dequant=False, quant_axis=qaxis,
                                     out_dtype=torch.float32)
                q = Parameter(data=lv.to(torch.int8), name=(wt.name or "w") + ".int8", trainable=False)
                q.stop_gradient = True
                sp = Parameter(data=s.float(), name=(wt.name or "w") + ".scale", trainable=False)
                sp.stop_gradient = True
                out = _new_var(blk, _wrap(wt._t.to("meta")), (wt.name or "w") + ".dequantized")
                dq = _make_op("dequantize_linear", {"x": q, "scale": sp, "bit_length": self._bits,
                                                    "quant_axis": qaxis if qaxis is not None else -1}, out)
                _insert_before(blk, op, dq)
                done[id(wt)] = out
            _replace_input(op, w, done[id(wt)])
        return _ret(graph, prog)


class TransformForMobilePass:
    """the reference renames fake_quantize_* / fake_dequantize_* ops to quantize / dequantize for
    Paddle-Lite; the ops here are already written as reference fake-quant types, which the mobile
    converters read, so the program is returned unchanged (kept for API parity)"""

    def __init__(self):
        pass

    def apply(self, graph):
        return graph


# ------------------------------------------------------------------------------------ out scale
class OutScaleForTrainingPass:
    """moving-average output-scale observers (moving_average_abs_max_scale) behind the outputs of
    the ops of ``_teller_set`` types"""

    def __init__(self, scope=None, place=None, moving_rate=0.9, is_test=None, scale_dict=None):
        self._rate = moving_rate
        self._is_test = is_test
        self._types = set(QUANT_OPS) | set(QDQ_OPS)

    def apply(self, graph):
        prog = _prog(graph)
        blk = prog.global_block()
        for op in list(blk.ops):
            typ = _ref_type(op)
            if typ not in self._types or P.is_train_op(op):
                continue
            outs = op.outputs if isinstance(op.outputs, (tuple, list)) else (op.outputs,)
            v = outs[0]
            if not isinstance(v, P.Variable) or not v._t.is_floating_point():
                continue
            obs = _make_op("moving_average_abs_max_scale",
                           {"x": v, "in_scale": _state(0.0, name="outscale.scale"),
                            "in_state": _state(0.0, name="outscale.state"), "in_accum": _state(0.0, name="outscale.accum"),
                            "moving_rate": self._rate, "is_test": bool(self._is_test)},
                           _new_var(blk, v, (v.name or "out") + ".outscale"))
            blk.ops.insert(blk.ops.index(op) + 1, obs)
            for o in P._iter_vars(obs.outputs):
                o.op = obs
            op.attrs["out_scale_observer"] = obs
        return _ret(graph, prog)


class OutScaleForInferencePass:
    """moves each observer's scale into its producer op's ``out_threshold`` attribute and removes
    the observer (the reference's inference-side counterpart)"""

    def __init__(self, scope=None):
        pass

    def apply(self, graph):
        prog = _prog(graph)
        blk = prog.global_block()
        keep = []
        for op in blk.ops:
            if _ref_type(op) == "moving_average_abs_max_scale":
                x = op.kwargs["x"]
                prod = getattr(x, "op", None)
                if prod is not None:
                    prod.attrs.setdefault("extra_attrs", {})["out_threshold"] = \
                        float(op.kwargs["in_scale"]._t.reshape(-1)[0].item())
                outs = op.outputs if isinstance(op.outputs, (tuple, list)) else (op.outputs,)
                for other in blk.ops:
                    for k, v in list(other.kwargs.items()):
                        if v is outs[0]:
                            _replace_input(other, k, x)
                continue
            keep.append(op)
        blk.ops = keep
        return _ret(graph, prog)


# ----------------------------------------------------------------------- quantize_linear (V2)
def _pair(blk, v, scale, bits, axis):
    """quantize_linear -> dequantize_linear on ``v`` (straight-through in training)"""
    q = _new_var(blk, v, (getattr(v, "name", "x") or "x") + ".quantized")
    d = _new_var(blk, v, (getattr(v, "name", "x") or "x") + ".dequantized")
    qop = _make_op("quantize_linear", {"x": v, "scale": scale, "bit_length": bits, "quant_axis": axis}, q)
    dop = _make_op("dequantize_linear", {"x": q, "scale": scale, "bit_length": bits, "quant_axis": axis}, d)
    return d, [qop, dop]


class QuantizationTransformPassV2(QuantizationTransformPass):
    """as QuantizationTransformPass, but written as quantize_linear / dequantize_linear pairs (the
    ONNX-style export format of the 2.4 reference); the activation scale is observed by a
    moving-average observer in training"""

    def apply(self, graph):
        prog = _prog(graph)
        blk = prog.global_block()
        from .....ops import quant as Q
        seen = {}
        for op, act, w, axis in _quantizable(prog, self._types, self._skip):
            v = op.kwargs[act]
            if isinstance(v, Tensor) and v._t.is_floating_point():
                if id(v) not in seen:
                    s = _state(0.001, name="quant.scale")
                    obs = _make_op("moving_average_abs_max_scale",
                                   {"x": v, "in_scale": s, "in_state": _state(1.0, name="quant.state"),
                                    "in_accum": _state(1.0, name="quant.accum"), "moving_rate": self._rate,
                                    "is_test": bool(self._is_test)}, _new_var(blk, v, "observed"))
                    obs_out = obs.outputs
                    _insert_before(blk, op, obs)
                    d, ops = _pair(blk, obs_out, s, self._abits, -1)
                    for o in ops:
                        _insert_before(blk, op, o)
                    seen[id(v)] = d
                _replace_input(op, act, seen[id(v)])
            if w is not None and _is_weight(op.kwargs[w]):
                wt = op.kwargs[w]
                if id(wt) not in seen:
                    ax = axis if self._wtype == "channel_wise_abs_max" else -1
                    sc = Q.channel_abs_max(wt._t, axis) if ax != -1 else Q.abs_max(wt._t)
                    sp = Parameter(data=sc.float(), name=(wt.name or "w") + ".quant_scale", trainable=False)
                    sp.stop_gradient = True
                    d, ops = _pair(blk, wt, sp, self._wbits, ax)
                    for o in ops:
                        _insert_before(blk, op, o)
                    seen[id(wt)] = d
                _replace_input(op, w, seen[id(wt)])
        return _ret(graph, prog)


class AddQuantDequantPassV2(AddQuantDequantPass):
    def apply(self, graph):
        prog = _prog(graph)
        blk = prog.global_block()
        cache = {}
        for op in list(blk.ops):
            ref = op_reference(op)
            if ref is None or ref[0] not in self._types or _skipped(op, self._skip) or P.is_train_op(op):
                continue
            for slot, k in ref[1].items():
                v = op.kwargs.get(k)
                if not isinstance(v, P.Variable) or not v._t.is_floating_point():
                    continue
                if id(v) not in cache:
                    s = _state(0.001, name="quant_dequant.scale")
                    obs = _make_op("moving_average_abs_max_scale",
                                   {"x": v, "in_scale": s, "in_state": _state(1.0, name="quant_dequant.state"),
                                    "in_accum": _state(1.0, name="quant_dequant.accum"), "moving_rate": self._rate,
                                    "is_test": bool(self._is_test)}, _new_var(blk, v, "observed"))
                    _insert_before(blk, op, obs)
                    d, ops = _pair(blk, obs.outputs, s, self._bits, -1)
                    for o in ops:
                        _insert_before(blk, op, o)
                    cache[id(v)] = d
                _replace_input(op, k, cache[id(v)])
        return _ret(graph, prog)


class ReplaceFakeQuantDequantPass:
    """fake_quantize_dequantize_* ops -> quantize_linear + dequantize_linear with the same scale"""

    def __init__(self, scope=None, place=None, quant_bits=8):
        self._bits = quant_bits

    def apply(self, graph):
        prog = _prog(graph)
        blk = prog.global_block()
        from .....ops import quant as Q
        new_ops = []
        for op in blk.ops:
            typ = _ref_type(op)
            if typ not in _FAKE_QDQ:
                new_ops.append(op)
                continue
            x = op.kwargs["x"]
            bits = op.kwargs.get("bit_length", self._bits)
            axis = -1
            if typ == "fake_quantize_dequantize_moving_average_abs_max":
                scale = op.kwargs["in_scale"]
            elif _is_weight(x):
                axis = op.kwargs.get("quant_axis", 0) if typ.startswith("fake_channel") else -1
                s = Q.channel_abs_max(x._t, axis) if axis != -1 else Q.abs_max(x._t)
                scale = Parameter(data=s.float(), name=_unique("quant_scale"), trainable=False)
                scale.stop_gradient = True
            else:
                new_ops.append(op)   # a dynamic per-batch abs-max on an activation: no fixed scale
                continue
            outs = op.outputs if isinstance(op.outputs, (tuple, list)) else (op.outputs,)
            d, pair = _pair(blk, x, scale, bits, axis)
            new_ops += pair
            for other in blk.ops:
                for k, v in list(other.kwargs.items()):
                    if v is outs[0]:
                        _replace_input(other, k, d)
        blk.ops = new_ops
        for op in new_ops:
            for v in P._iter_vars(op.outputs):
                v.op = op
        return _ret(graph, prog)


class QuantWeightPass:
    """weights of a quantize_linear / dequantize_linear program stored as int8 levels; only the
    dequantize_linear op stays in front of the consumer"""

    def __init__(self, scope=None, place=None, bias_correction=False, quant_bits=8, save_int_weight=True):
        self._bits = quant_bits

    def apply(self, graph):
        prog = _prog(graph)
        blk = prog.global_block()
        from .....ops import quant as Q
        keep = []
        qmap = {}
        for op in blk.ops:
            if _ref_type(op) == "quantize_linear" and _is_weight(op.kwargs["x"]):
                x, s = op.kwargs["x"], op.kwargs["scale"]
                ax = op.kwargs.get("quant_axis", -1)
                lv = Q.quant_dequant(x._t, s._t, op.kwargs.get("bit_length", self._bits), 0, dequant=False,
                                     quant_axis=ax if s._t.numel() > 1 else None, out_dtype=torch.float32)
                p = Parameter(data=lv.to(torch.int8), name=(x.name or "w") + ".int8", trainable=False)
                p.stop_gradient = True
                outs = op.outputs if isinstance(op.outputs, (tuple, list)) else (op.outputs,)
                qmap[id(outs[0])] = p
                continue
            keep.append(op)
        for op in keep:
            for k, v in list(op.kwargs.items()):
                if id(v) in qmap:
                    _replace_input(op, k, qmap[id(v)])
        blk.ops = keep
        return _ret(graph, prog)
