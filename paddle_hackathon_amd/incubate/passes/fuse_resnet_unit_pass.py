"""Fuse conv2d -> batch_norm (-> elementwise_add) -> relu chains of a static Program into
``resnet_unit`` ops (reference: python/paddle/incubate/passes/fuse_resnet_unit_pass.py:49 — the
conv+bn+relu and conv+bn+conv+bn+add+relu patterns; the op: incubate/operators/resnet_unit.py).

Three patterns, matched on the recorded ops (each intermediate read by exactly the next op of the
chain, bias-free non-grouped convolutions, inference or training batch norm):

    relu(bn(conv(x)))                       -> resnet_unit(x)
    relu(bn(conv(x)) + z)                   -> resnet_unit(x, z, fuse_add=True)
    relu(bn(conv(x)) + bn'(conv'(z)))       -> resnet_unit(x, z, has_shortcut=True)
      (both convolutions with the same kernel size / padding)

On the MI355X kernels the rewrite removes one full read + write of the activation per unit: the
BN normalise, the residual add and the ReLU become one batch_norm.hip pass, and the convolution's
epilogue already reduces the BN statistics."""
from __future__ import annotations

__all__ = ["fuse_resnet_unit"]

_CONV = "nn.functional.conv.conv2d"
_BN = "nn.functional.norm.batch_norm"
_ADD = "tensor.math.add"
_RELU = "nn.functional.activation.relu"


def _short(op):
    t = op.type
    return t[len("paddle_hackathon_amd."):] if t.startswith("paddle_hackathon_amd.") else t


def _consumers(ops):
    from ...static import program as P
    n = {}
    for op in ops:
        for v in P._iter_vars((op.args, op.kwargs)):
            n[id(v)] = n.get(id(v), 0) + 1
    return n


def _single(out):
    from ...static import program as P
    vs = list(P._iter_vars(out))
    return vs[0] if len(vs) == 1 else None


def _conv_ok(op):
    k = op.kwargs
    return (_short(op) == _CONV and not op.args and k.get("bias") is None and k.get("groups", 1) == 1
            and k.get("data_format", "NCHW") in ("NCHW", "NHWC"))


def fuse_resnet_unit(program, keep=()):
    """rewrite ``program``'s global block in place; ``keep``: Variables that must stay materialised
    (fetch targets). Returns the number of units formed."""
    from ...static import program as P
    from ..operators.resnet_unit import resnet_unit
    blk = program.global_block()
    keep_ids = {id(v) for v in keep}
    fused = 0
    changed = True
    while changed:
        changed = False
        ops = blk.ops
        uses = _consumers(ops)
        producer = {}
        for i, op in enumerate(ops):
            for v in P._iter_vars(op.outputs):
                producer[id(v)] = i

        def only_reader(v):
            return v is not None and uses.get(id(v), 0) == 1 and id(v) not in keep_ids

        def conv_bn(v):
            """(conv index, bn index) when v is bn(conv(.)) with single-reader intermediates"""
            j = producer.get(id(v))
            if j is None or _short(ops[j]) != _BN or ops[j].args:
                return None
            c = ops[j].kwargs.get("x")
            i = producer.get(id(c)) if c is not None else None
            if i is None or not _conv_ok(ops[i]) or not only_reader(_single(ops[i].outputs)):
                return None
            if ops[j].kwargs.get("data_format", "NCHW") != ops[i].kwargs.get("data_format", "NCHW"):
                return None
            return i, j

        for r, op in enumerate(ops):
            if _short(op) != _RELU or op.args:
                continue
            src = op.kwargs.get("x")
            if not only_reader(src):
                continue
            z, short, main = None, None, None
            k = producer.get(id(src))
            if k is None:
                continue
            if _short(ops[k]) == _ADD and not ops[k].args:
                a, b = ops[k].kwargs.get("x"), ops[k].kwargs.get("y")
                if not (isinstance(a, P.Variable) and isinstance(b, P.Variable)):
                    continue
                for first, second in ((a, b), (b, a)):
                    cb = conv_bn(first) if only_reader(first) else None
                    if cb is None:
                        continue
                    sc = conv_bn(second) if only_reader(second) else None
                    if sc is not None and ops[sc[0]].kwargs["weight"].shape[2:] == ops[cb[0]].kwargs["weight"].shape[2:] \
                            and ops[sc[0]].kwargs.get("padding") == ops[cb[0]].kwargs.get("padding"):
                        main, short = cb, sc
                    elif tuple(second.shape) == tuple(_single(ops[cb[1]].outputs).shape):
                        main, z = cb, second
                    if main is not None:
                        break
                if main is None:
                    continue
                chain = [main[0], main[1], k, r] + (list(short) if short else [])
            else:
                main = conv_bn(src)
                if main is None:
                    continue
                chain = [main[0], main[1], r]
            cv, bn = ops[main[0]].kwargs, ops[main[1]].kwargs
            fmt = cv.get("data_format", "NCHW")
            training = bool(bn.get("training", False))
            kw = dict(x=cv["x"], filter_x=cv["weight"], scale_x=bn["weight"], bias_x=bn["bias"],
                      mean_x=bn["running_mean"], var_x=bn["running_var"], z=None, filter_z=None, scale_z=None,
                      bias_z=None, mean_z=None, var_z=None, stride=cv.get("stride", 1), stride_z=1,
                      padding=cv.get("padding", 0), dilation=cv.get("dilation", 1), groups=1,
                      momentum=bn.get("momentum", 0.9), eps=bn.get("epsilon", 1e-5), data_format=fmt,
                      fuse_add=z is not None, has_shortcut=short is not None,
                      use_global_stats=bool(bn.get("use_global_stats") or False), is_test=not training,
                      act="relu", filter_layout="OIHW")
            if z is not None:
                kw["z"] = z
            if short is not None:
                cz, bz = ops[short[0]].kwargs, ops[short[1]].kwargs
                kw.update(z=cz["x"], filter_z=cz["weight"], scale_z=bz["weight"], bias_z=bz["bias"],
                          mean_z=bz["running_mean"], var_z=bz["running_var"], stride_z=cz.get("stride", 1))
            new = P.OpDesc(f"{resnet_unit.__module__}.resnet_unit", resnet_unit, (), kw, op.outputs,
                           attrs={"fused_from": [ops[i].type for i in chain]})
            for v in P._iter_vars(op.outputs):
                v.op = new
            # the unit runs where the relu was (all its inputs exist there); the chain's ops go
            ops[r] = new
            for i in sorted(set(chain) - {r}, reverse=True):
                del ops[i]
            fused += 1
            changed = True
            break
    return fused


def _register():
    from ...parallel.passes import PassBase, register_pass

    @register_pass("fuse_resnet_unit")
    class FuseResNetUnitPass(PassBase):
        def _check_self(self):
            return True

        def _check_conflict(self, other_pass):
            return True

        def _apply_single_impl(self, main_program, startup_program, context):
            n = fuse_resnet_unit(main_program, keep=self.get_attr("keep", ()) or ())
            context.set_attr("fuse_resnet_unit_count", n)
    return FuseResNetUnitPass


FuseResNetUnitPass = _register()
