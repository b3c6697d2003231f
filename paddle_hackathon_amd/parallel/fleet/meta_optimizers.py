"""Fleet meta-optimizers for dygraph collective training (reference:
python/paddle/distributed/fleet/meta_optimizers/{gradient_merge,localsgd,dgc,fp16_allreduce,lars,
lamb}_optimizer.py, which rewrite a static Program; fluid/optimizer.py LarsMomentumOptimizer and
DGCMomentumOptimizer, operators/dgc_op.h).

``fleet.distributed_optimizer`` applies them from the DistributedStrategy flags:

* ``lars`` / ``lamb``: the inner Momentum / Adam(W) is replaced by LARS momentum / LAMB.
* ``fp16_allreduce``: fp32 gradient buckets are all-reduced in bf16 (MI355X: bf16 keeps fp32's
  exponent range, so no loss scaling is needed for the collective) and cast back.
* ``dgc``: top-k gradient sparsification with momentum correction and factor masking after
  ``rampup_begin_step``; ranks exchange (index, value) pairs with all_gather instead of the
  dense all-reduce.
* ``localsgd`` / ``adaptive_localsgd``: ranks step locally and average parameters every k steps
  (adaptive: k = ceil(sqrt(lr0 * loss / (lr * loss0) * init_k)), clipped to [1, 16]).
* ``gradient_merge``: gradients accumulate over ``k_steps`` micro-batches (the data-parallel
  all-reduce runs only on the last one) before the inner step; ``avg`` divides by k.
"""
from __future__ import annotations

import math

import torch
import torch.distributed as dist

from ...framework.core import Tensor
from ...optimizer.optimizer import Optimizer
from .. import collective as C

__all__ = ["LarsMomentumOptimizer", "GradientMergeOptimizer", "LocalSGDOptimizer", "DGCMomentumOptimizer",
           "apply_meta_optimizers"]


class LarsMomentumOptimizer(Optimizer):
    """Momentum with layer-wise adaptive rate scaling:
    local_lr = lr * lars_coeff * ||w|| / (||g|| + lars_weight_decay * ||w|| + epsilon);
    v = mu * v + local_lr * (g + lars_weight_decay * w); w -= v."""

    def __init__(self, learning_rate=0.001, momentum=0.9, lars_coeff=0.001, lars_weight_decay=0.0005,
                 parameters=None, grad_clip=None, exclude_from_weight_decay=None, epsilon=0.0,
                 multi_precision=False, rescale_grad=1.0, name=None):
        super().__init__(learning_rate, parameters, None, grad_clip, name, multi_precision)
        self._momentum = momentum
        self._lars_coeff = float(lars_coeff)
        self._lars_wd = float(lars_weight_decay)
        self._exclude = list(exclude_from_weight_decay or [])
        self._epsilon = float(epsilon)
        self._rescale_grad = float(rescale_grad)

    def _update(self, pgs):
        lr = self.get_lr()
        for p, g, group in pgs:
            m = self._master(p)
            w = m._t if m is not None else p._t
            gt = g._t.float() * self._rescale_grad
            wd = 0.0 if any(e in (p.name or "") for e in self._exclude) else self._lars_wd
            wn, gn = w.float().norm(), gt.norm()
            local = torch.where((wn > 0) & (gn > 0),
                                lr * self._lr_ratio(p, group) * self._lars_coeff * wn / (gn + wd * wn + self._epsilon),
                                torch.full_like(wn, lr * self._lr_ratio(p, group)))
            v = self._acc("velocity", p)._t
            v.mul_(self._momentum).add_(local * (gt + wd * w.float()))
            w.sub_(v.to(w.dtype))
            if m is not None:
                p._t.copy_(m._t)


_dp_model_hook = [lambda: None]   # set by fleet: the DataParallel model of the job, if any


class _Wrapper:
    def __init__(self, inner):
        self._inner_opt = inner

    @property
    def _dpm(self):
        return self._dp if self._dp is not None else _dp_model_hook[0]()

    def clear_grad(self, set_to_zero=True):
        self._inner_opt.clear_grad(set_to_zero)

    def minimize(self, loss, startup_program=None, parameters=None, no_grad_set=None):
        self._last_loss = loss
        self.step()

    def __getattr__(self, item):
        return getattr(self._inner_opt, item)

    def _params(self):
        return [p for p in self._inner_opt._parameter_list if not p.stop_gradient]


class GradientMergeOptimizer(_Wrapper):
    """Accumulate gradients over ``k_steps`` calls of step(); the inner optimizer runs on the k-th
    (gradients divided by k when ``avg``). With a DataParallel model the all-reduce is skipped on
    the first k-1 micro-batches (its reducer is told not to sync) and sums the accumulated grads
    once."""

    def __init__(self, inner, k_steps=1, avg=True, dp_model=None):
        super().__init__(inner)
        self.k_steps = max(1, int(k_steps))
        self.avg = bool(avg)
        self._dp = dp_model
        self._count = 0
        self._set_sync()

    def _set_sync(self):
        dp = self._dpm
        if dp is not None and hasattr(dp, "_grad_need_sync"):
            dp._grad_need_sync = (self._count + 1) % self.k_steps == 0

    def step(self):
        self._count += 1
        if self._count % self.k_steps == 0:
            if self.avg and self.k_steps > 1:
                with torch.no_grad():
                    for p in self._params():
                        if p._t.grad is not None:
                            p._t.grad.div_(self.k_steps)
            self._inner_opt.step()
            self._inner_opt.clear_grad(set_to_zero=False)
        self._set_sync()

    def clear_grad(self, set_to_zero=True):
        pass   # gradients are cleared after the merged step


class LocalSGDOptimizer(_Wrapper):
    """Local steps with periodic parameter averaging (k fixed, or adaptive from the loss)."""

    def __init__(self, inner, k_steps=1, begin_step=1, dp_model=None, group=None, adaptive=False, init_k_steps=1):
        super().__init__(inner)
        self.k_steps = max(1, int(init_k_steps if adaptive else k_steps))
        self.init_k = max(1, int(init_k_steps))
        self.begin_step = int(begin_step)
        self.adaptive = adaptive
        self._dp = dp_model
        self._pg = C._resolve_group(group)
        self._n = C.get_world_size(group) if group is not None else C.get_world_size()
        self._step = 0
        self._last_sync = 0
        self._loss0 = self._lr0 = None
        self._last_loss = None
        self._set_sync()

    def _set_sync(self):
        dp = self._dpm
        if dp is not None and hasattr(dp, "_grad_need_sync"):
            # up to begin_step: synchronous data parallel (gradient all-reduce every step)
            dp._grad_need_sync = self._step + 1 <= self.begin_step

    def _average(self):
        if self._n <= 1 or not C.is_initialized():
            return
        with torch.no_grad():
            for p in self._params():
                t = p._t
                dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self._pg)
                t.div_(self._n)
                m = self._inner_opt._master(p) if hasattr(self._inner_opt, "_master") else None
                if m is not None:
                    m._t.copy_(t.float())

    def _loss_value(self):
        l = self._last_loss
        if l is None:
            return None
        v = l._t if isinstance(l, Tensor) else l
        v = v.detach().float().reshape(-1)[0:1].clone()
        if self._n > 1 and C.is_initialized():
            dist.all_reduce(v, op=dist.ReduceOp.SUM, group=self._pg)
            v /= self._n
        return float(v)

    def step(self):
        self._inner_opt.step()
        self._step += 1
        if self._step > self.begin_step and self._step - self._last_sync >= self.k_steps:
            self._average()
            self._last_sync = self._step
            if self.adaptive:
                loss = self._loss_value()
                lr = float(self._inner_opt.get_lr())
                if loss is not None and self._loss0 is None:
                    self._loss0, self._lr0 = loss, lr
                elif loss is not None and self._loss0 and lr > 0:
                    k = math.ceil(math.sqrt(self._lr0 * loss / (lr * self._loss0) * self.init_k))
                    self.k_steps = min(16, max(1, k))
        self._set_sync()


class DGCMomentumOptimizer(_Wrapper):
    """Deep gradient compression (Lin et al. 2018; reference DGCMomentumOptimizer): per tensor
    u = m u + g, v += u, send the top (1 - sparsity) |v| entries (all_gather of indices and
    values), zero them in u and v; the averaged sparse gradient updates the parameter with plain
    SGD (momentum already lives in u). Dense momentum + all-reduce before rampup_begin_step and
    for tensors under ``min_numel`` elements."""

    def __init__(self, inner, rampup_begin_step=0, rampup_step=1, sparsity=(0.999,), dp_model=None, group=None,
                 min_numel=1024):
        super().__init__(inner)
        self.momentum = float(getattr(inner, "_momentum", 0.9))
        self.begin = int(rampup_begin_step)
        self.rampup = max(1, int(rampup_step))
        self.sparsity = list(sparsity) or [0.999]
        self.min_numel = int(min_numel)
        self._dp = dp_model
        self._pg = C._resolve_group(group)
        self._n = C.get_world_size(group) if group is not None else C.get_world_size()
        self._step = 0
        self._u, self._v = {}, {}
        self._no_dp_sync()

    def _no_dp_sync(self):
        dp = self._dpm
        if dp is not None and hasattr(dp, "_grad_need_sync"):
            dp._grad_need_sync = False   # this optimizer does the communication

    def current_sparsity(self):
        if self._step < self.begin:
            return 0.0
        i = min(len(self.sparsity) - 1, (self._step - self.begin) * len(self.sparsity) // self.rampup)
        return float(self.sparsity[i])

    def _allreduce_dense(self, g):
        if self._n > 1 and C.is_initialized():
            dist.all_reduce(g, op=dist.ReduceOp.SUM, group=self._pg)
            g.div_(self._n)

    def _sparse_exchange(self, p, g, sparsity):
        key = id(p)
        gf = g.float().reshape(-1)
        u = self._u.setdefault(key, torch.zeros_like(gf))
        v = self._v.setdefault(key, torch.zeros_like(gf))
        u.mul_(self.momentum).add_(gf)
        v.add_(u)
        k = max(1, int(round(gf.numel() * (1.0 - sparsity))))
        idx = v.abs().topk(k, sorted=False).indices
        vals = v[idx]
        u[idx] = 0
        v[idx] = 0
        dense = torch.zeros_like(gf)
        if self._n > 1 and C.is_initialized():
            all_idx = [torch.empty_like(idx) for _ in range(self._n)]
            all_val = [torch.empty_like(vals) for _ in range(self._n)]
            dist.all_gather(all_idx, idx, group=self._pg)
            dist.all_gather(all_val, vals, group=self._pg)
            for i_, v_ in zip(all_idx, all_val):
                dense.index_add_(0, i_, v_)
            dense.div_(self._n)
        else:
            dense.index_add_(0, idx, vals)
        return dense.reshape(g.shape).to(g.dtype)

    def step(self):
        self._no_dp_sync()
        sparsity = self.current_sparsity()
        lr = float(self._inner_opt.get_lr())
        with torch.no_grad():
            if sparsity <= 0.0:
                for p in self._params():
                    if p._t.grad is not None:
                        self._allreduce_dense(p._t.grad)
                self._inner_opt.step()
            else:
                dense_params = []
                for p in self._params():
                    g = p._t.grad
                    if g is None:
                        continue
                    if g.numel() < self.min_numel:
                        self._allreduce_dense(g)
                        dense_params.append(p)
                        continue
                    sg = self._sparse_exchange(p, g, sparsity)
                    m = self._inner_opt._master(p) if hasattr(self._inner_opt, "_master") else None
                    target = m._t if m is not None else p._t
                    target.sub_((lr * sg.float()).to(target.dtype))
                    if m is not None:
                        p._t.copy_(m._t)
                    p._t.grad = None
                if dense_params:
                    self._inner_opt.step()
        self._step += 1


def apply_meta_optimizers(optimizer, strategy, dp_model=None, group=None):
    """Wrap ``optimizer`` as the strategy asks (see module docstring). Returns the new optimizer."""
    from ...optimizer.optimizer import Adam, Lamb, Momentum
    opt = optimizer
    params = opt._parameter_list
    if strategy.lars and isinstance(opt, Momentum):
        c = strategy.lars_configs
        opt = LarsMomentumOptimizer(opt._learning_rate, opt._momentum, c.get("lars_coeff", 0.001),
                                    c.get("lars_weight_decay", 0.0005), parameters=params, grad_clip=opt._grad_clip,
                                    exclude_from_weight_decay=c.get("exclude_from_weight_decay"),
                                    epsilon=c.get("epsilon", 0.0))
    elif strategy.lamb and isinstance(opt, Adam):
        c = strategy.lamb_configs
        excl = list(c.get("exclude_from_weight_decay") or [])
        opt = Lamb(opt._learning_rate, c.get("lamb_weight_decay", 0.01), opt._beta1, opt._beta2, opt._epsilon,
                   parameters=params, grad_clip=opt._grad_clip,
                   exclude_from_weight_decay_fn=(lambda p: any(e in (p.name or "") for e in excl)) if excl else None)
    if strategy.fp16_allreduce and dp_model is not None and getattr(dp_model, "_reducer", None) is not None:
        dp_model._reducer.comm_dtype = torch.bfloat16
    return opt


def wrap_meta_optimizers(opt, strategy, dp_model=None, group=None):
    """The stepping wrappers (applied outside the hybrid-parallel optimizer)."""
    if strategy.dgc and isinstance(getattr(opt, "_inner_opt", opt), Optimizer) and hasattr(
            getattr(opt, "_inner_opt", opt), "_momentum"):
        c = strategy.dgc_configs
        opt = DGCMomentumOptimizer(opt, c.get("rampup_begin_step", 0), c.get("rampup_step", 1),
                                   c.get("sparsity", [0.999]), dp_model=dp_model, group=group)
    elif strategy.adaptive_localsgd:
        c = getattr(strategy, "adaptive_localsgd_configs", None) or {"init_k_steps": 1, "begin_step": 1}
        opt = LocalSGDOptimizer(opt, begin_step=c.get("begin_step", 1), dp_model=dp_model, group=group,
                                adaptive=True, init_k_steps=c.get("init_k_steps", 1))
    elif strategy.localsgd:
        c = strategy.localsgd_configs
        opt = LocalSGDOptimizer(opt, c.get("k_steps", 1), c.get("begin_step", 1), dp_model=dp_model, group=group)
    if strategy.gradient_merge:
        c = strategy.gradient_merge_configs
        opt = GradientMergeOptimizer(opt, c.get("k_steps", 1), c.get("avg", True), dp_model=dp_model)
    return opt
