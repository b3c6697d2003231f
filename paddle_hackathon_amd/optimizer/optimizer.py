"""Optimizers (reference: python/paddle/optimizer/{optimizer,sgd,momentum,adam,adamw,adamax,
adagrad,adadelta,rmsprop,lamb}.py; kernels phi/kernels/gpu/{adam,adamw,momentum,...}_kernel.cu).

Adam/AdamW/Momentum/SGD update *every* parameter with one multi-tensor HIP
launch per (param dtype, grad dtype) group (ops.fused_adam_ / fused_momentum_),
with fp32 master weights for bf16/fp16 parameters (``multi_precision``).
Accumulator names follow the reference (``linear_0.w_0_moment1_0`` …) so optimizer
checkpoints (.pdopt) keep the same keys; a restore is strict (see ``set_state_dict``).
"""
from __future__ import annotations

import collections
import math
import re
import warnings

import numpy as np
import torch

from ..framework.core import Tensor, Parameter, _wrap
from ..framework import core as _core
from ..regularizer import L1Decay, L2Decay, WeightDecayRegularizer
from .. import ops as _ops
from .lr import LRScheduler
from ..utils import unique_name

__all__ = ["Optimizer", "SGD", "Momentum", "Adam", "AdamW", "Adamax", "Adagrad", "Adadelta", "RMSProp", "Lamb"]


class Optimizer:
    def __init__(self, learning_rate=0.001, parameters=None, weight_decay=None, grad_clip=None, name=None,
                 multi_precision=True):
        if parameters is not None and isinstance(parameters, Tensor):
            raise TypeError("parameters should be a list of Tensor / dict")
        self._parameter_list = None
        self._param_groups = []
        if parameters is not None:
            parameters = list(parameters)
            if parameters and isinstance(parameters[0], dict):
                for g in parameters:
                    self._add_param_group(dict(g))
            else:
                self._add_param_group({"params": parameters})
            self._parameter_list = [p for g in self._param_groups for p in g["params"]]
        self._learning_rate = learning_rate
        if isinstance(weight_decay, (int, float)):
            self.regularization = L2Decay(float(weight_decay)) if weight_decay else None
        else:
            self.regularization = weight_decay
        self._grad_clip = grad_clip
        self._name = name
        self._multi_precision = multi_precision
        self._accumulators = collections.defaultdict(dict)   # acc_name -> {param.name: Tensor}
        self._master_weights = {}
        self._step_count = 0
        self._state_loaded = {}

    # -- groups ----------------------------------------------------------------------
    def _add_param_group(self, group):
        params = group["params"]
        if isinstance(params, Tensor):
            params = [params]
        group["params"] = list(params)
        self._param_groups.append(group)

    @property
    def _parameters(self):
        return self._parameter_list

    # -- lr -----------------------------------------------------------------------------
    def get_lr(self):
        lr = self._learning_rate
        return float(lr()) if isinstance(lr, LRScheduler) else float(lr)

    def set_lr(self, value):
        if isinstance(self._learning_rate, LRScheduler):
            raise RuntimeError("optimizer's learning rate can't be LRScheduler when invoke this API")
        self._learning_rate = float(value)
        for t in self.__dict__.get("_lr_devs", {}).values():   # graph-captured steps read these
            t.fill_(float(value))

    def set_lr_scheduler(self, scheduler):
        self._learning_rate = scheduler

    # -- accumulators ---------------------------------------------------------------
    _STATE_META = ("master_weights", "LR_Scheduler", "@step_count@")

    def _loaded_accs(self):
        return [k for k in self._state_loaded if k not in self._STATE_META]

    def _take_loaded(self, base, key):
        """the loaded value of accumulator ``key`` (= ``unique_name.generate(base)``); a saved
        name with another generator suffix (``base_N``: the saving process had created more
        optimizers over the same parameters) is taken when it is the only one"""
        if key in self._state_loaded:
            return self._state_loaded.pop(key)
        pat = re.compile(re.escape(base) + r"_\d+$")
        hits = [k for k in self._state_loaded if pat.match(k)]
        if len(hits) == 1:
            return self._state_loaded.pop(hits[0])
        return None

    def _acc_base(self, pname, name):
        # an optimizer created with name="opt" prefixes its accumulators (optimizer.py:623-624)
        return f"{pname}_{self._name}_{name}" if self._name else f"{pname}_{name}"

    def _acc(self, name, p, dtype=torch.float32, fill=0.0, shape=None):
        """accumulator ``name`` of parameter ``p``, named as the reference's _add_accumulator names
        it — ``unique_name.generate(f"{param.name}_{name}")``, e.g. ``linear_0.w_0_moment1_0``
        (python/paddle/optimizer/optimizer.py:636). Once a state dict is loaded, every accumulator
        created must come from it: a missing one raises as the reference's assertion does
        (optimizer.py:656-659) instead of silently restarting from ``fill``."""
        d = self._accumulators[name]
        t = d.get(p.name)
        if t is None:
            base = self._acc_base(p.name, name)
            key = unique_name.generate(base)
            src = self._take_loaded(base, key) if self._state_loaded else None
            if src is None and self.__dict__.get("_strict_acc"):
                raise AssertionError(f"Optimizer set error, {key} should in state dict")
            if src is not None:
                src_t = src._t if isinstance(src, Tensor) else torch.as_tensor(np.asarray(src))
                t = _wrap(src_t.to(device=p._t.device, dtype=dtype).clone())
                if shape is None and tuple(t._t.shape) != tuple(p._t.shape):
                    raise ValueError(f"accumulator {key}: loaded shape {tuple(t._t.shape)} != parameter "
                                     f"{p.name} shape {tuple(p._t.shape)}")
            else:
                shp = p._t.shape if shape is None else shape
                t = _wrap(torch.full(shp, fill, dtype=dtype, device=p._t.device))
            t.name = key
            t.persistable = True
            d[p.name] = t
        return t

    def _master(self, p):
        if not self._multi_precision or p._t.dtype not in (torch.float16, torch.bfloat16):
            return None
        m = self._master_weights.get(p.name)
        if m is None:
            mw = self._state_loaded.get("master_weights", {})
            if p.name in mw:
                src = mw[p.name]
                src_t = src._t if isinstance(src, Tensor) else torch.as_tensor(np.asarray(src))
                m = _wrap(src_t.to(device=p._t.device, dtype=torch.float32).clone())
            else:
                m = _wrap(p._t.detach().float().clone())
            m.name = unique_name.generate(p.name + "_fp32_master")
            self._master_weights[p.name] = m
        return m

    # -- step ---------------------------------------------------------------------------
    def _collect(self):
        out = []
        for g in self._param_groups:
            for p in g["params"]:
                if p.stop_gradient or p._t.grad is None:
                    continue
                out.append((p, _wrap(p._t.grad), g))
        return out

    def _apply_clip(self, pgs):
        self._gscale_dev = None
        if self._grad_clip is None:
            return
        from ..nn.clip import ClipGradByGlobalNorm
        import os
        if type(self._grad_clip) is ClipGradByGlobalNorm and getattr(self, "_fuses_grad_scale", False) and pgs \
                and os.environ.get("PHA_FUSED_CLIP", "1") != "0" \
                and all(p._t.is_cuda for p, _, _ in pgs) \
                and all(p.need_clip if hasattr(p, "need_clip") else True for p, _, _ in pgs):
            # global-norm clip folded into the fused optimizer kernel: it multiplies the factor in
            # as it reads each gradient (no extra read + write pass over all gradients)
            self._gscale_dev = self._grad_clip.scale_factor([(p, g) for p, g, _ in pgs])
            return
        self._grad_clip([(p, g) for p, g, _ in pgs])

    def _wd_for(self, p, group):
        reg = p.regularizer if getattr(p, "regularizer", None) is not None else group.get("weight_decay", self.regularization)
        if isinstance(reg, (int, float)):
            return float(reg), "l2"
        if isinstance(reg, L2Decay):
            return reg.coeff, "l2"
        if isinstance(reg, L1Decay):
            return reg.coeff, "l1"
        return 0.0, None

    def step(self):
        if self._parameter_list is None:
            raise ValueError("parameters must be given in dygraph mode")
        pgs = self._collect()
        self._apply_clip(pgs)
        self._step_count += 1
        with torch.no_grad():
            self._update(pgs)
        if getattr(self._learning_rate, "_auto_step", False):   # schedules that step with the optimizer
            self._learning_rate.step()

    def _update(self, pgs):
        raise NotImplementedError

    def _lr_ratio(self, p, group):
        r = p.optimize_attr.get("learning_rate", 1.0) if hasattr(p, "optimize_attr") else 1.0
        if "learning_rate" in group:
            r *= float(group["learning_rate"])
        return r

    def minimize(self, loss, startup_program=None, parameters=None, no_grad_set=None):
        if not _core.in_dynamic_mode():
            from ..static.program import minimize_static
            return minimize_static(self, loss, parameters, no_grad_set)
        if parameters is not None and self._parameter_list is None:
            self._add_param_group({"params": list(parameters)})
            self._parameter_list = list(parameters)
        self.step()
        return None, [(p, _wrap(p._t.grad)) for p in (self._parameter_list or []) if p._t.grad is not None]

    def clear_grad(self, set_to_zero=True):
        ps = [p for p in self._parameter_list or [] if p._t.grad is not None]
        if set_to_zero:
            if ps:
                torch._foreach_zero_([p._t.grad for p in ps])
        else:
            for p in ps:
                p._t.grad = None

    clear_gradients = clear_grad

    def backward(self, loss, startup_program=None, parameters=None, no_grad_set=None, callbacks=None):
        loss.backward()
        return [(p, _wrap(p._t.grad)) for p in (self._parameter_list or []) if p._t.grad is not None]

    def apply_gradients(self, params_grads):
        self.step()

    # -- state -------------------------------------------------------------------------
    def state_dict(self):
        sd = {}
        for name, d in self._accumulators.items():
            for pname, t in d.items():
                sd[t.name] = t
        if self._master_weights:
            sd["master_weights"] = dict(self._master_weights)
        if isinstance(self._learning_rate, LRScheduler):
            sd["LR_Scheduler"] = self._learning_rate.state_dict()
        sd["@step_count@"] = self._step_count
        return sd

    def set_state_dict(self, state_dict):
        """Restore accumulators / master weights / LR state (reference optimizer.py:310). Keys are
        the reference's accumulator names; accumulators that exist are overwritten now, the rest
        are taken when first created — and from then on every accumulator must be in the dict
        (AssertionError otherwise, as the reference). Keys that belong to no parameter of this
        optimizer are reported (a renamed model restored nothing for them)."""
        state_dict = dict(state_dict)
        if isinstance(self._learning_rate, LRScheduler) and "LR_Scheduler" in state_dict:
            self._learning_rate.set_state_dict(state_dict.pop("LR_Scheduler"))
        self._step_count = int(state_dict.pop("@step_count@", self._step_count))
        self.__dict__.pop("_pstep", None)   # per-parameter counts are re-read from the loaded beta-pow accumulators
        for name, d in self._accumulators.items():
            for pname, t in d.items():
                base = self._acc_base(pname, name)
                v = state_dict.pop(t.name, None)
                if v is None:
                    pat = re.compile(re.escape(base) + r"_\d+$")
                    hits = [k for k in state_dict if pat.match(k)]
                    v = state_dict.pop(hits[0]) if len(hits) == 1 else None
                if v is None:
                    raise AssertionError(f"Optimizer set error, {t.name} should in state dict")
                src = v._t if isinstance(v, Tensor) else torch.as_tensor(np.asarray(v))
                with torch.no_grad():
                    t._t.copy_(src.to(t._t.device, t._t.dtype).reshape(t._t.shape))
        mw = state_dict.get("master_weights")
        if mw:
            for pname, m in list(self._master_weights.items()):
                if pname in mw:
                    v = mw[pname]
                    src = v._t if isinstance(v, Tensor) else torch.as_tensor(np.asarray(v))
                    with torch.no_grad():
                        m._t.copy_(src.to(m._t.device, torch.float32))
        names = sorted({p.name for g in self._param_groups for p in g["params"]}, key=len, reverse=True)
        stray = [k for k in state_dict if k not in self._STATE_META and not any(k.startswith(n + "_") for n in names)]
        if stray and names:
            warnings.warn(f"optimizer state: {len(stray)} key(s) match no parameter of this optimizer and are "
                          f"ignored (e.g. {stray[:3]}); parameter names look like {names[-1]!r}", stacklevel=2)
            for k in stray:
                state_dict.pop(k)
        # snapshot the rest (loaded lazily on first use): the caller's dict may hold live tensors
        # of another optimizer that keep changing after this call
        snap = {}
        for k, v in state_dict.items():
            if isinstance(v, Tensor):
                snap[k] = _wrap(v._t.detach().clone())
            elif isinstance(v, dict):
                snap[k] = {kk: (_wrap(vv._t.detach().clone()) if isinstance(vv, Tensor) else vv) for kk, vv in v.items()}
            else:
                snap[k] = v
        self._state_loaded.update(snap)
        self._strict_acc = bool(self._loaded_accs())

    set_dict = set_state_dict


class SGD(Optimizer):
    def __init__(self, learning_rate=0.001, parameters=None, weight_decay=None, grad_clip=None, multi_precision=False, name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name, multi_precision)

    def _update(self, pgs):
        lr = self.get_lr()
        for p, g, group in pgs:
            wd, kind = self._wd_for(p, group)
            gt = g._t.float()
            m = self._master(p)
            target = m._t if m is not None else p._t
            if kind == "l2":
                gt = gt + wd * target.float()
            elif kind == "l1":
                gt = gt + wd * torch.sign(target.float())
            target.add_(gt.to(target.dtype), alpha=-lr * self._lr_ratio(p, group))
            if m is not None:
                p._t.copy_(m._t)


class Momentum(Optimizer):
    def __init__(self, learning_rate=0.001, momentum=0.9, parameters=None, use_nesterov=False, weight_decay=None,
                 grad_clip=None, multi_precision=False, rescale_grad=1.0, name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name, multi_precision)
        self._momentum = momentum
        self._use_nesterov = bool(use_nesterov)
        self._rescale_grad = rescale_grad

    def _update(self, pgs):
        lr = self.get_lr()
        params, grads, vels, masters, ratios, wds = [], [], [], [], [], []
        for p, g, group in pgs:
            wd, kind = self._wd_for(p, group)
            if kind == "l1":
                g._t.add_(torch.sign(p._t) * wd)
                wd = 0.0
            params.append(p._t)
            grads.append(g._t)
            vels.append(self._acc("velocity", p)._t)
            m = self._master(p)
            masters.append(None if m is None else m._t)
            ratios.append(self._lr_ratio(p, group))
            wds.append(wd)
        if params:
            if params[0].is_cuda:
                from ..ops import hip
                hip.multi_tensor_momentum(params, grads, vels, masters, lr, self._momentum, self._use_nesterov, 0.0,
                                          ratios, self._rescale_grad, wds)
            else:
                for i in range(len(params)):
                    _ops.fused_momentum_([params[i]], [grads[i]], [vels[i]], [masters[i]], lr, self._momentum,
                                         self._use_nesterov, wds[i], [ratios[i]], self._rescale_grad)


class Adam(Optimizer):
    _decoupled = False

    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-08, parameters=None, weight_decay=None,
                 grad_clip=None, lazy_mode=False, multi_precision=True, name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name, multi_precision)
        self._beta1 = float(beta1._t.item()) if isinstance(beta1, Tensor) else float(beta1)
        self._beta2 = float(beta2._t.item()) if isinstance(beta2, Tensor) else float(beta2)
        self._epsilon = float(epsilon._t.item()) if isinstance(epsilon, Tensor) else float(epsilon)
        self._lazy_mode = lazy_mode
        self._grad_scale = 1.0
        self._fuses_grad_scale = True   # _update feeds the clip factor to the multi-tensor kernel

    def _decay_for(self, p, group):
        wd, kind = self._wd_for(p, group)
        return wd, kind

    def _update(self, pgs):
        lr = self.get_lr()
        params, grads, m1, m2, masters, ratios, wds = [], [], [], [], [], [], []
        step_pows = []
        if getattr(self, "_gscale_dev", None) is not None and \
                any(self._decay_for(p, group)[1] == "l1" for p, _, group in pgs):
            # L1 decay is added to the CLIPPED gradient: apply the clip factor up front instead
            by_dt = {}
            for _, g, _ in pgs:
                by_dt.setdefault(g._t.dtype, []).append(g._t)
            for dt, gs in by_dt.items():
                torch._foreach_mul_(gs, self._gscale_dev.to(dt))
            self._gscale_dev = None
        for p, g, group in pgs:
            wd, kind = self._decay_for(p, group)
            if kind == "l1":
                g._t.add_(torch.sign(p._t) * wd)
                wd = 0.0
            params.append(p._t)
            grads.append(g._t)
            m1.append(self._acc("moment1", p)._t)
            m2.append(self._acc("moment2", p)._t)
            b1p = self._acc("beta1_pow_acc", p, fill=self._beta1, shape=[1])
            b2p = self._acc("beta2_pow_acc", p, fill=self._beta2, shape=[1])
            step_pows.append((b1p, b2p))
            m = self._master(p)
            masters.append(None if m is None else m._t)
            ratios.append(self._lr_ratio(p, group))
            wds.append(wd)
        if not params:
            return
        # Bias correction is per parameter, as the reference's beta1_pow_acc / beta2_pow_acc
        # (adam_kernel.cu): a parameter that got no gradient in some steps (unused embedding rows'
        # table, an idle MoE expert) or state resumed from a reference .pdopt keeps its own count.
        # The count lives on the host (no device sync per step); it is recovered once from the
        # beta1_pow accumulator value (beta1^(t+1) after t updates) for parameters it has not seen.
        steps = self._param_steps([p for p, _, _ in pgs], step_pows)
        groups = {}
        for i, st in enumerate(steps):   # one launch per (update index, device): host-offloaded and
            groups.setdefault((st, params[i].device), []).append(i)   # device parameters may mix
        capturing = torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()
        for (step, dev), idx in groups.items():
            sel = (lambda xs: [xs[i] for i in idx]) if len(groups) > 1 else (lambda xs: xs)
            if dev.type == "cuda":
                from ..ops import hip
                lr_dev = pow_dev = None
                if not capturing:
                    self._lr_device(dev, lr)   # exists before any capture (its creation is no graph node)
                else:
                    # a hipGraph replays this launch: learning rate and bias corrections come from
                    # device scalars (the scheduler refreshes the former, the beta-pow accumulators
                    # advance in-graph), as the reference's adam kernel reads LearningRate /
                    # Beta1Pow / Beta2Pow tensors
                    lr_dev = self._lr_device(dev, lr)
                    b1p, b2p = step_pows[idx[0]]
                    pow_dev = (b1p._t, b2p._t)
                hip.multi_tensor_adam(sel(params), sel(grads), sel(m1), sel(m2), sel(masters), lr, self._beta1,
                                      self._beta2, self._epsilon, step, 0.0, self._decoupled, sel(ratios),
                                      self._grad_scale, sel(wds), gscale_dev=getattr(self, "_gscale_dev", None),
                                      lr_dev=lr_dev, pow_dev=pow_dev)
            else:
                for i in idx:
                    _ops.fused_adam_([params[i]], [grads[i]], [m1[i]], [m2[i]], [masters[i]], lr, self._beta1,
                                     self._beta2, self._epsilon, step, wds[i], self._decoupled, [ratios[i]],
                                     self._grad_scale)
        torch._foreach_mul_([b[0]._t for b in step_pows], self._beta1)
        torch._foreach_mul_([b[1]._t for b in step_pows], self._beta2)

    def _lr_device(self, dev, lr):
        """fp32 device scalar holding the learning rate, refreshed by the LR scheduler's step() /
        set_lr() outside any capture (a replayed graph reads it)"""
        cache = self.__dict__.setdefault("_lr_devs", {})
        t = cache.get(dev)
        if t is None:
            t = torch.full((1,), float(lr), dtype=torch.float32, device=dev)
            cache[dev] = t
            if isinstance(self._learning_rate, LRScheduler):
                self._learning_rate._register_device_lr(t)
        return t

    def _param_steps(self, params, pows):
        """1-based update index of every parameter for this step (host counters). A count not seen
        yet is read back once from the beta-pow accumulators (beta^(t+1) after t updates; beta2's
        decays slower, so it is preferred while it has not underflowed)."""
        cnt = self.__dict__.setdefault("_pstep", {})
        missing = [i for i, p in enumerate(params) if p.name not in cnt]
        if missing:
            vals = torch.stack([torch.stack([pows[i][0]._t.reshape(()).float().cpu(),
                                             pows[i][1]._t.reshape(()).float().cpu()]) for i in missing]).tolist()
            for i, (v1, v2) in zip(missing, vals):
                t = None
                for beta, v in ((self._beta2, v2), (self._beta1, v1)):
                    if 0.0 < beta < 1.0 and v > 0.0:
                        t = int(round(math.log(v) / math.log(beta))) - 1
                        break
                cnt[params[i].name] = max(0, self._step_count - 1 if t is None else t)
        out = []
        for p in params:
            cnt[p.name] += 1
            out.append(cnt[p.name])
        return out


class AdamW(Adam):
    _decoupled = True

    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8, parameters=None, weight_decay=0.01,
                 lr_ratio=None, apply_decay_param_fun=None, grad_clip=None, lazy_mode=False, multi_precision=True, name=None):
        super().__init__(learning_rate, beta1, beta2, epsilon, parameters, None, grad_clip, lazy_mode, multi_precision, name)
        self._coeff = float(weight_decay) if not isinstance(weight_decay, WeightDecayRegularizer) else weight_decay.coeff
        self._apply_decay_param_fun = apply_decay_param_fun
        self._lr_ratio_fn = lr_ratio

    def _decay_for(self, p, group):
        coeff = group.get("weight_decay", self._coeff)
        if isinstance(coeff, WeightDecayRegularizer):
            coeff = coeff.coeff
        if self._apply_decay_param_fun is not None and not self._apply_decay_param_fun(p.name):
            return 0.0, None
        return float(coeff), "decoupled"

    def _lr_ratio(self, p, group):
        r = super()._lr_ratio(p, group)
        if self._lr_ratio_fn is not None:
            r *= float(self._lr_ratio_fn(p))
        return r


class Adamax(Optimizer):
    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-08, parameters=None, weight_decay=None,
                 grad_clip=None, name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name, False)
        self._beta1, self._beta2, self._epsilon = beta1, beta2, epsilon

    def _update(self, pgs):
        lr = self.get_lr()
        for p, g, group in pgs:
            wd, kind = self._wd_for(p, group)
            gt = g._t.float() + (wd * p._t.float() if kind == "l2" else 0)
            m = self._acc("moment", p)._t
            u = self._acc("inf_norm", p)._t
            b1p = self._acc("beta1_pow_acc", p, fill=self._beta1, shape=[1])._t
            m.mul_(self._beta1).add_(gt, alpha=1 - self._beta1)
            torch.maximum(u * self._beta2, gt.abs() + self._epsilon, out=u)
            lr_t = lr * self._lr_ratio(p, group) / (1 - b1p)
            p._t.sub_((lr_t * m / u).to(p._t.dtype))
            b1p.mul_(self._beta1)


class Adagrad(Optimizer):
    def __init__(self, learning_rate, epsilon=1e-06, parameters=None, weight_decay=None, grad_clip=None, name=None,
                 initial_accumulator_value=0.0):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name, False)
        self._epsilon, self._init_acc = epsilon, initial_accumulator_value

    def _update(self, pgs):
        lr = self.get_lr()
        for p, g, group in pgs:
            wd, kind = self._wd_for(p, group)
            gt = g._t.float() + (wd * p._t.float() if kind == "l2" else 0)
            m = self._acc("moment", p, fill=self._init_acc)._t
            m.add_(gt * gt)
            p._t.sub_((lr * self._lr_ratio(p, group) * gt / (m.sqrt() + self._epsilon)).to(p._t.dtype))


class Adadelta(Optimizer):
    def __init__(self, learning_rate=0.001, epsilon=1.0e-6, rho=0.95, parameters=None, weight_decay=None, grad_clip=None, name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name, False)
        self._epsilon, self._rho = epsilon, rho

    def _update(self, pgs):
        lr = self.get_lr()
        for p, g, group in pgs:
            wd, kind = self._wd_for(p, group)
            gt = g._t.float() + (wd * p._t.float() if kind == "l2" else 0)
            sg = self._acc("_avg_squared_grad", p)._t
            su = self._acc("_avg_squared_update", p)._t
            sg.mul_(self._rho).add_(gt * gt, alpha=1 - self._rho)
            upd = -torch.sqrt((su + self._epsilon) / (sg + self._epsilon)) * gt
            su.mul_(self._rho).add_(upd * upd, alpha=1 - self._rho)
            p._t.add_((lr * self._lr_ratio(p, group) * upd).to(p._t.dtype))


class RMSProp(Optimizer):
    def __init__(self, learning_rate, rho=0.95, epsilon=1.0e-6, momentum=0.0, centered=False, parameters=None,
                 weight_decay=None, grad_clip=None, name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name, False)
        self._rho, self._epsilon, self._momentum, self._centered = rho, epsilon, momentum, centered

    def _update(self, pgs):
        lr = self.get_lr()
        for p, g, group in pgs:
            wd, kind = self._wd_for(p, group)
            gt = g._t.float() + (wd * p._t.float() if kind == "l2" else 0)
            ms = self._acc("mean_square", p)._t
            mom = self._acc("momentum", p)._t
            ms.mul_(self._rho).add_(gt * gt, alpha=1 - self._rho)
            if self._centered:
                mg = self._acc("mean_grad", p)._t
                mg.mul_(self._rho).add_(gt, alpha=1 - self._rho)
                denom = ms - mg * mg + self._epsilon
            else:
                denom = ms + self._epsilon
            mom.mul_(self._momentum).add_(lr * self._lr_ratio(p, group) * gt / denom.sqrt())
            p._t.sub_(mom.to(p._t.dtype))


class Lamb(Optimizer):
    def __init__(self, learning_rate=0.001, lamb_weight_decay=0.01, beta1=0.9, beta2=0.999, epsilon=1e-6, parameters=None,
                 grad_clip=None, exclude_from_weight_decay_fn=None, multi_precision=False, name=None):
        super().__init__(learning_rate, parameters, None, grad_clip, name, multi_precision)
        self._wd, self._beta1, self._beta2, self._epsilon = lamb_weight_decay, beta1, beta2, epsilon
        self._exclude = exclude_from_weight_decay_fn

    def _update(self, pgs):
        lr = self.get_lr()
        for p, g, group in pgs:
            gt = g._t.float()
            m = self._master(p)
            w = (m._t if m is not None else p._t).float()
            m1 = self._acc("moment1", p)._t
            m2 = self._acc("moment2", p)._t
            b1p = self._acc("beta1_pow_acc", p, fill=self._beta1, shape=[1])._t
            b2p = self._acc("beta2_pow_acc", p, fill=self._beta2, shape=[1])._t
            m1.mul_(self._beta1).add_(gt, alpha=1 - self._beta1)
            m2.mul_(self._beta2).addcmul_(gt, gt, value=1 - self._beta2)
            mhat = m1 / (1 - b1p)
            vhat = m2 / (1 - b2p)
            wd = 0.0 if (self._exclude is not None and self._exclude(p)) else self._wd
            r = mhat / (vhat.sqrt() + self._epsilon) + wd * w
            wn, rn = w.norm(), r.norm()
            trust = torch.where((wn > 0) & (rn > 0), wn / rn, torch.ones_like(wn))
            neww = w - lr * self._lr_ratio(p, group) * trust * r
            if m is not None:
                m._t.copy_(neww)
            p._t.copy_(neww.to(p._t.dtype))
            b1p.mul_(self._beta1)
            b2p.mul_(self._beta2)
