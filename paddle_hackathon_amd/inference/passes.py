"""Inference IR passes over a static Program (reference: paddle/fluid/inference/api/
paddle_pass_builder.cc:156-176 GpuPassStrategy, framework/ir/conv_bn_fuse_pass.cc, fc_fuse_pass.cc,
skip_layernorm_fuse_pass.cc, multihead_matmul_fuse_pass.cc, delete_dropout_op_pass.cc,
identity_scale_op_clean_pass.cc, constant_folding_pass.cc, auto_mixed_precision_pass.cc).

Our Programs record ops at API granularity (``conv2d``, ``batch_norm``, ``linear``, ``matmul``,
``softmax`` ...), so each pass is a pattern match over producer/consumer links of one block
followed by a rewrite into a fused op from ``inference/fused_ops.py`` (whose HIP paths are the
fused kernels of ops/fused.py and the flash-attention kernels). A rewritten op takes over the
output Variables of the last op of its pattern, so consumers and fetch targets stay bound.
Every pass returns how many rewrites it made; ``PassStrategy`` is the ordered, editable list
(``Config.pass_builder()``, ``Config.delete_pass``).
"""
from __future__ import annotations

import torch

from ..framework.core import Parameter, Tensor, _wrap
from ..static import program as P
from ..static.program import OpDesc, Variable, _iter_vars, prune_ops
from . import fused_ops as FO

_PKG = "paddle_hackathon_amd."
CONV2D = _PKG + "nn.functional.conv.conv2d"
BN = _PKG + "nn.functional.norm.batch_norm"
BN_ACT = _PKG + "nn.functional.norm.batch_norm_act"
LINEAR = _PKG + "nn.functional.common.linear"
MATMUL = _PKG + "tensor.math.matmul"
ADD = _PKG + "tensor.math.add"
MULTIPLY = _PKG + "tensor.math.multiply"
SCALE = _PKG + "tensor.math.scale"
SOFTMAX = _PKG + "nn.functional.activation.softmax"
DROPOUT = _PKG + "nn.functional.common.dropout"
LAYER_NORM = _PKG + "nn.functional.norm.layer_norm"
ACTS = {_PKG + "nn.functional.activation.relu": "relu", _PKG + "nn.functional.activation.gelu": "gelu"}


def _qual(fn):
    return f"{fn.__module__}.{fn.__name__}"


class _Graph:
    """producer / consumer index of one block's ops (Variables by identity)"""

    def __init__(self, ops, protected):
        self.ops = ops
        self.protected = {id(v) for v in protected}
        self.producer, self.consumers = {}, {}
        for op in ops:
            for v in _iter_vars(op.outputs):
                self.producer[id(v)] = op
            for v in _iter_vars((op.args, op.kwargs, op.attrs.get("captured", []))):
                self.consumers.setdefault(id(v), []).append(op)

    def only_consumer(self, v, op):
        """``op`` is the single reader of ``v`` and ``v`` is not fetched"""
        return id(v) not in self.protected and self.consumers.get(id(v), []) == [op]

    def next_op(self, v):
        c = self.consumers.get(id(v), [])
        return c[0] if len(c) == 1 and id(v) not in self.protected else None


def _single_out(op):
    return op.outputs if isinstance(op.outputs, Variable) else None


def _replace_in_tree(tree, old, new):
    if tree is old:
        return new
    if isinstance(tree, list):
        return [_replace_in_tree(t, old, new) for t in tree]
    if isinstance(tree, tuple):
        return tuple(_replace_in_tree(t, old, new) for t in tree)
    if isinstance(tree, dict):
        return {k: _replace_in_tree(v, old, new) for k, v in tree.items()}
    return tree


def _rebind(ops, old, new, fetches):
    """every read of Variable ``old`` now reads ``new`` (identity-op removal)"""
    for op in ops:
        op.args = _replace_in_tree(op.args, old, new)
        op.kwargs = _replace_in_tree(op.kwargs, old, new)
        if op.exec is not None:
            for k in ("captured", "true_outs", "false_outs", "body_outs", "cond_out", "pred"):
                if k in op.attrs:
                    op.attrs[k] = _replace_in_tree(op.attrs[k], old, new)
    for i, f in enumerate(fetches):
        if f is old:
            fetches[i] = new


def _fused(fn, kwargs, outputs):
    op = OpDesc(_qual(fn), fn, (), kwargs, outputs)
    for v in _iter_vars(outputs):
        v.op = op
    return op


def _const(x):
    return isinstance(x, Tensor) and not isinstance(x, Variable)


# ------------------------------------------------------------------------------------------ passes
class Pass:
    name = "pass"

    def apply(self, program, fetches):
        n = 0
        for blk in program.blocks:
            n += self.apply_block(blk, fetches)
        return n

    def apply_block(self, blk, fetches):
        return 0


class DeleteDropoutPass(Pass):
    """inference dropout: ``upscale_in_train`` is the identity, ``downscale_in_infer`` a scale"""
    name = "delete_dropout_op_pass"

    def apply_block(self, blk, fetches):
        n = 0
        for op in list(blk.ops):
            if op.type != DROPOUT or op.kwargs.get("training", True) and not getattr(blk.program, "_is_test", False):
                continue
            out, x = _single_out(op), op.kwargs.get("x")
            if out is None or not isinstance(x, Tensor):
                continue
            if op.kwargs.get("mode", "upscale_in_train") == "downscale_in_infer":
                p = float(op.kwargs.get("p", 0.5))
                new = _fused(FO.scale_inference, {"x": x, "scale": 1.0 - p}, out)
                blk.ops[blk.ops.index(op)] = new
            else:
                blk.ops.remove(op)
                _rebind([o for b in blk.program.blocks for o in b.ops], out, x, fetches)
            n += 1
        return n


class IdentityScaleCleanPass(Pass):
    name = "identity_scale_op_clean_pass"

    def apply_block(self, blk, fetches):
        n = 0
        for op in list(blk.ops):
            if op.type == SCALE and float(op.kwargs.get("scale", 1.0)) == 1.0 and float(op.kwargs.get("bias", 0.0)) == 0.0:
                out, x = _single_out(op), op.kwargs.get("x")
                if out is not None and isinstance(x, Tensor) and not isinstance(op.kwargs.get("scale"), Tensor):
                    blk.ops.remove(op)
                    _rebind([o for b in blk.program.blocks for o in b.ops], out, x, fetches)
                    n += 1
        return n


class ConstantFoldingPass(Pass):
    """ops whose tensor inputs are all constants (parameters included) run once at optimisation
    time; their outputs become constants"""
    name = "constant_folding_pass"

    def apply_block(self, blk, fetches):
        n = 0
        for op in list(blk.ops):
            if op.exec is not None or op.fn is None or P.is_train_op(op):
                continue
            ins = list(_iter_vars((op.args, op.kwargs)))
            tens = [t for t in _iter_tensors_all((op.args, op.kwargs))]
            if ins or not tens:
                continue
            out = _single_out(op)
            if out is None or op.type in (DROPOUT,):
                continue
            with torch.no_grad():
                val = op.fn(*op.args, **op.kwargs)
            if not isinstance(val, Tensor):
                continue
            blk.ops.remove(op)
            _rebind([o for b in blk.program.blocks for o in b.ops], out, _wrap(val._t.detach()), fetches)
            n += 1
        return n


def _iter_tensors_all(tree):
    if isinstance(tree, Tensor):
        yield tree
    elif isinstance(tree, (list, tuple)):
        for t in tree:
            yield from _iter_tensors_all(t)
    elif isinstance(tree, dict):
        for t in tree.values():
            yield from _iter_tensors_all(t)


class ConvBNFusePass(Pass):
    """conv2d -> batch_norm(inference) folds BN into the conv weights / bias; a ``batch_norm_act``
    (BN + residual add + ReLU) becomes ``conv2d_fusion`` with the residual and activation"""
    name = "conv_bn_fuse_pass"

    def apply_block(self, blk, fetches):
        n = 0
        g = _Graph(blk.ops, fetches)
        for conv in list(blk.ops):
            if conv.type != CONV2D:
                continue
            out = _single_out(conv)
            bn = g.next_op(out) if out is not None else None
            if bn is None or bn.type not in (BN, BN_ACT) or bn.kwargs.get("x") is not out:
                continue
            kw = bn.kwargs
            if kw.get("training", False) and not kw.get("use_global_stats"):
                continue
            w, b = conv.kwargs.get("weight"), conv.kwargs.get("bias")
            stats = [kw.get(k) for k in ("running_mean", "running_var", "weight", "bias")]
            if not _const(w) or (b is not None and not _const(b)) or not all(s is None or _const(s) for s in stats[:2]) \
                    or stats[0] is None or stats[1] is None:
                continue
            mean, var, gamma, beta = (None if s is None else s._t.float() for s in stats)
            eps = float(kw.get("epsilon", 1e-5))
            s = torch.rsqrt(var + eps) * (gamma if gamma is not None else 1.0)
            wt = w._t.float() * s.reshape(-1, *([1] * (w._t.dim() - 1)))
            bt = ((b._t.float() if b is not None else torch.zeros_like(mean)) - mean) * s
            if beta is not None:
                bt = bt + beta
            nw = Parameter(data=wt.to(w._t.dtype), name=f"{w.name}.bn_folded")
            nb = Parameter(data=bt.to(w._t.dtype), name=f"{w.name}.bn_folded_bias")
            ckw = dict(conv.kwargs, weight=nw, bias=nb)
            residual, act = kw.get("residual"), kw.get("act")
            if residual is None and act is None:
                new = OpDesc(conv.type, conv.fn, conv.args, ckw, bn.outputs)
                for v in _iter_vars(bn.outputs):
                    v.op = new
            else:
                new = _fused(FO.conv2d_fusion, dict(ckw, residual=residual, act=act), bn.outputs)
            blk.ops[blk.ops.index(conv)] = new
            blk.ops.remove(bn)
            g = _Graph(blk.ops, fetches)
            n += 1
        return n


class ConvElementwiseAddActPass(Pass):
    """conv2d(+bias) -> add(residual) -> relu  =>  conv2d_fusion"""
    name = "conv_elementwise_add_act_fuse_pass"

    def apply_block(self, blk, fetches):
        n = 0
        g = _Graph(blk.ops, fetches)
        for conv in list(blk.ops):
            if conv.type != CONV2D:
                continue
            out = _single_out(conv)
            nxt = g.next_op(out) if out is not None else None
            residual, last = None, conv
            if nxt is not None and nxt.type == ADD:
                other = nxt.kwargs.get("y") if nxt.kwargs.get("x") is out else nxt.kwargs.get("x")
                if isinstance(other, Tensor) and tuple(other._t.shape) == tuple(out._t.shape):
                    residual, last = other, nxt
                    nxt = g.next_op(_single_out(nxt))
            if nxt is None or ACTS.get(nxt.type) != "relu":
                continue
            new = _fused(FO.conv2d_fusion, dict(conv.kwargs, residual=residual, act="relu"), nxt.outputs)
            # at the activation's position: the residual may come from an op after the conv (the
            # other branch of a block: conv -> add(other_conv_bn, conv) -> relu)
            blk.ops[blk.ops.index(nxt)] = new
            if last is not conv:
                blk.ops.remove(last)
            blk.ops.remove(conv)
            g = _Graph(blk.ops, fetches)
            n += 1
        return n


class FCFusePass(Pass):
    """matmul(x, W) -> add(b) => linear; linear -> relu/gelu => fc with the activation in the
    GEMM epilogue / bias-act kernel"""
    name = "fc_fuse_pass"

    def apply_block(self, blk, fetches):
        n = 0
        g = _Graph(blk.ops, fetches)
        for op in list(blk.ops):
            if op not in blk.ops:
                continue
            if op.type == MATMUL and _const(op.kwargs.get("y")) and op.kwargs.get("y")._t.dim() == 2 \
                    and not op.kwargs.get("transpose_x") and not op.kwargs.get("transpose_y"):
                out = _single_out(op)
                nxt = g.next_op(out) if out is not None else None
                if nxt is not None and nxt.type == ADD:
                    other = nxt.kwargs.get("y") if nxt.kwargs.get("x") is out else nxt.kwargs.get("x")
                    if _const(other) and other._t.dim() == 1:
                        new = _fused(FO.fc, {"x": op.kwargs["x"], "weight": op.kwargs["y"], "bias": other}, nxt.outputs)
                        blk.ops[blk.ops.index(op)] = new
                        blk.ops.remove(nxt)
                        g = _Graph(blk.ops, fetches)
                        n += 1
                        op = new
            if op.type in (LINEAR, _qual(FO.fc)) and not op.kwargs.get("activation"):
                out = _single_out(op)
                nxt = g.next_op(out) if out is not None else None
                if nxt is not None and nxt.type in ACTS and nxt.kwargs.get("x") is out \
                        and not nxt.kwargs.get("approximate", False):
                    kw = {"x": op.kwargs["x"], "weight": op.kwargs["weight"], "bias": op.kwargs.get("bias"),
                          "activation": ACTS[nxt.type]}
                    new = _fused(FO.fc, kw, nxt.outputs)
                    blk.ops[blk.ops.index(op)] = new
                    blk.ops.remove(nxt)
                    g = _Graph(blk.ops, fetches)
                    n += 1
        return n


class SkipLayerNormFusePass(Pass):
    """add(x, residual) -> layer_norm  =>  one fused residual-add + LayerNorm kernel"""
    name = "skip_layernorm_fuse_pass"

    def apply_block(self, blk, fetches):
        n = 0
        g = _Graph(blk.ops, fetches)
        for op in list(blk.ops):
            if op.type != ADD or op not in blk.ops:
                continue
            out = _single_out(op)
            ln = g.next_op(out) if out is not None else None
            x, y = op.kwargs.get("x"), op.kwargs.get("y")
            if ln is None or ln.type != LAYER_NORM or ln.kwargs.get("x") is not out or not isinstance(x, Tensor) \
                    or not isinstance(y, Tensor) or tuple(x._t.shape) != tuple(y._t.shape):
                continue
            ns = ln.kwargs.get("normalized_shape")
            ns = [ns] if isinstance(ns, int) else list(ns)
            if len(ns) != 1:
                continue
            new = _fused(FO.skip_layernorm, {"x": x, "y": y, "weight": ln.kwargs.get("weight"),
                                             "bias": ln.kwargs.get("bias"), "epsilon": ln.kwargs.get("epsilon", 1e-5)},
                         ln.outputs)
            blk.ops[blk.ops.index(op)] = new
            blk.ops.remove(ln)
            g = _Graph(blk.ops, fetches)
            n += 1
        return n


class MultiHeadMatmulFusePass(Pass):
    """matmul(q, k^T) -> scale -> [add mask] -> softmax -> [dropout(eval)] -> matmul(., v)
    => fused attention on the flash kernels ([B, H, S, D] operands)"""
    name = "multihead_matmul_fuse_pass"

    def apply_block(self, blk, fetches):
        n = 0
        g = _Graph(blk.ops, fetches)
        for qk in list(blk.ops):
            if qk not in blk.ops or qk.type != MATMUL or not qk.kwargs.get("transpose_y") or qk.kwargs.get("transpose_x"):
                continue
            chain, cur = [qk], _single_out(qk)
            scale, mask = 1.0, None
            nxt = g.next_op(cur) if cur is not None else None
            if nxt is not None and nxt.type == SCALE and float(nxt.kwargs.get("bias", 0.0)) == 0.0 \
                    and not isinstance(nxt.kwargs.get("scale"), Tensor):
                scale = float(nxt.kwargs.get("scale", 1.0))
                chain.append(nxt)
                cur = _single_out(nxt)
                nxt = g.next_op(cur)
            elif nxt is not None and nxt.type == MULTIPLY:
                other = nxt.kwargs.get("y") if nxt.kwargs.get("x") is cur else nxt.kwargs.get("x")
                if isinstance(other, (int, float)) or (_const(other) and other._t.numel() == 1):
                    scale = float(other) if isinstance(other, (int, float)) else float(other._t.reshape(-1)[0])
                    chain.append(nxt)
                    cur = _single_out(nxt)
                    nxt = g.next_op(cur)
            if nxt is not None and nxt.type == ADD:
                mask = nxt.kwargs.get("y") if nxt.kwargs.get("x") is cur else nxt.kwargs.get("x")
                chain.append(nxt)
                cur = _single_out(nxt)
                nxt = g.next_op(cur)
            if nxt is None or nxt.type != SOFTMAX or nxt.kwargs.get("axis", -1) not in (-1, 3):
                continue
            chain.append(nxt)
            cur = _single_out(nxt)
            nxt = g.next_op(cur)
            if nxt is not None and nxt.type == DROPOUT and not nxt.kwargs.get("training", True) \
                    and nxt.kwargs.get("mode", "upscale_in_train") == "upscale_in_train":
                chain.append(nxt)
                cur = _single_out(nxt)
                nxt = g.next_op(cur)
            if nxt is None or nxt.type != MATMUL or nxt.kwargs.get("x") is not cur or nxt.kwargs.get("transpose_x") \
                    or nxt.kwargs.get("transpose_y"):
                continue
            q, k, v = qk.kwargs.get("x"), qk.kwargs.get("y"), nxt.kwargs.get("y")
            if not all(isinstance(t, Tensor) and t._t.dim() == 4 for t in (q, k, v)):
                continue
            chain.append(nxt)
            new = _fused(FO.multihead_attention, {"q": q, "k": k, "v": v, "mask": mask, "scale": scale}, nxt.outputs)
            blk.ops[blk.ops.index(qk)] = new
            for o in chain[1:]:
                blk.ops.remove(o)
            g = _Graph(blk.ops, fetches)
            n += 1
        return n


class DeadCodeEliminationPass(Pass):
    name = "dead_code_elimination_pass"

    def apply(self, program, fetches):
        blk = program.global_block()
        before = len(blk.ops)
        if any(isinstance(f, Variable) for f in fetches):
            blk.ops = prune_ops(blk.ops, [f for f in fetches if isinstance(f, Variable)])
        return before - len(blk.ops)


class AutoMixedPrecisionPass(Pass):
    """weights of GEMM/conv-type ops to bf16 (or fp16); LayerNorm / BatchNorm / softmax keep fp32
    parameters (the kernels take fp32 scale/shift). Feeds are cast on entry by the predictor."""
    name = "auto_mixed_precision_pass"
    KEEP_FP32 = (LAYER_NORM, BN, BN_ACT, _PKG + "inference.fused_ops.skip_layernorm")

    def __init__(self, dtype=torch.bfloat16, black_list=()):
        self.dtype = dtype
        self.black = set(black_list)

    def apply(self, program, fetches):
        keep = set()
        for b in program.blocks:
            for op in b.ops:
                short = op.type.rsplit(".", 1)[-1]
                if op.type in self.KEEP_FP32 or short in self.black:
                    keep.update(id(t) for t in _iter_tensors_all((op.args, op.kwargs)))
        n = 0
        with torch.no_grad():
            for p in program.all_parameters():
                if p._t.is_floating_point() and id(p) not in keep and p._t.dtype != self.dtype:
                    p._t = p._t.to(self.dtype)
                    n += 1
            for v in program.global_block().vars.values():   # float feeds enter in the program's dtype
                if getattr(v, "is_data", False) and v._t.is_floating_point() and v._t.dtype != self.dtype:
                    v._t = torch.empty(tuple(v._t.shape), dtype=self.dtype, device="meta")
        program._amp_dtype = self.dtype
        return n


_PASSES = {c.name: c for c in (DeleteDropoutPass, IdentityScaleCleanPass, ConstantFoldingPass, ConvBNFusePass,
                               ConvElementwiseAddActPass, FCFusePass, SkipLayerNormFusePass, MultiHeadMatmulFusePass,
                               DeadCodeEliminationPass, AutoMixedPrecisionPass)}

GPU_PASSES = ["delete_dropout_op_pass", "identity_scale_op_clean_pass", "constant_folding_pass", "conv_bn_fuse_pass",
              "conv_elementwise_add_act_fuse_pass", "multihead_matmul_fuse_pass", "skip_layernorm_fuse_pass",
              "fc_fuse_pass", "dead_code_elimination_pass"]


class PassStrategy:
    """ordered pass list (reference paddle_pass_builder.h PaddlePassBuilder)"""

    def __init__(self, passes=None):
        self._passes = list(GPU_PASSES if passes is None else passes)
        self._debug = False

    def all_passes(self):
        return list(self._passes)

    def append_pass(self, name):
        self._passes.append(name)

    def insert_pass(self, idx, name):
        self._passes.insert(idx, name)

    def delete_pass(self, name):
        self._passes = [p for p in self._passes if p != name]

    def clear_passes(self):
        self._passes = []

    def turn_on_debug(self):
        self._debug = True

    def run(self, program, fetches, amp_dtype=None, black_list=()):
        stats = {}
        for name in self._passes:
            cls = _PASSES.get(name)
            if cls is None:
                raise KeyError(f"unknown IR pass {name!r}; known: {sorted(_PASSES)}")
            stats[name] = cls().apply(program, fetches)
        if amp_dtype is not None:
            stats[AutoMixedPrecisionPass.name] = AutoMixedPrecisionPass(amp_dtype, black_list).apply(program, fetches)
        if self._debug:
            print("[ir] " + ", ".join(f"{k}={v}" for k, v in stats.items()))
        return stats


def optimize_program(program, fetches, passes=None, amp_dtype=None):
    """apply the pass pipeline in place; ``fetches`` (list) is updated when a fetched Variable is
    rebound. -> {pass name: rewrites}"""
    return PassStrategy(passes).run(program, fetches, amp_dtype)
