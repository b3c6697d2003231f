"""High-level API: ``paddle.Model`` + summary/flops (reference: python/paddle/hapi/{model,
model_summary,static_flops,dynamic_flops}.py)."""
from __future__ import annotations

import os
import time

import numpy as np
import torch

from ..framework.core import Tensor, _wrap, to_tensor
from ..framework.io import save as _save, load as _load
from ..nn.layer.layers import Layer
from .. import io as _io
from . import callbacks as cbks_mod
from .callbacks import config_callbacks

__all__ = ["Model", "summary", "flops", "callbacks"]
callbacks = cbks_mod


def _to_list(x):
    if x is None:
        return []
    return list(x) if isinstance(x, (list, tuple)) else [x]


class Model:
    def __init__(self, network, inputs=None, labels=None):
        self.network = network
        self._inputs = inputs
        self._labels = labels
        self._optimizer = None
        self._loss = None
        self._metrics = []
        self._amp_level = "O0"
        self._scaler = None
        self.stop_training = False

    def prepare(self, optimizer=None, loss=None, metrics=None, amp_configs=None):
        self._optimizer = optimizer
        self._loss = loss
        self._metrics = _to_list(metrics)
        if amp_configs:
            from .. import amp
            level = amp_configs if isinstance(amp_configs, str) else amp_configs.get("level", "O1")
            self._amp_level = level
            if level != "O0":
                self._scaler = amp.GradScaler(init_loss_scaling=(amp_configs.get("init_loss_scaling", 2 ** 15)
                                                                 if isinstance(amp_configs, dict) else 2 ** 15))

    def _forward(self, inputs):
        if self._amp_level != "O0":
            from .. import amp
            with amp.auto_cast(level=self._amp_level):
                return self.network(*inputs)
        return self.network(*inputs)

    def train_batch(self, inputs, labels=None, update=True):
        self.network.train()
        inputs, labels = _to_list(inputs), _to_list(labels)
        outs = _to_list(self._forward([_as_t(x) for x in inputs]))
        losses = _to_list(self._loss(*(outs + [_as_t(l) for l in labels]))) if self._loss else outs
        total = losses[0]
        for l in losses[1:]:
            total = total + l
        if self._scaler is not None:
            self._scaler.scale(total).backward()
            if update:
                self._scaler.step(self._optimizer)
                self._scaler.update()
        else:
            total.backward()
            if update:
                self._optimizer.step()
        if update:
            self._optimizer.clear_grad()
        metrics = self._update_metrics(outs, labels)
        lv = [float(l.numpy()) for l in losses]
        return (lv, metrics) if metrics else lv

    def eval_batch(self, inputs, labels=None):
        self.network.eval()
        inputs, labels = _to_list(inputs), _to_list(labels)
        with torch.no_grad():
            outs = _to_list(self._forward([_as_t(x) for x in inputs]))
            losses = _to_list(self._loss(*(outs + [_as_t(l) for l in labels]))) if self._loss and labels else []
        metrics = self._update_metrics(outs, labels)
        lv = [float(l.numpy()) for l in losses]
        return (lv, metrics) if metrics else lv

    def predict_batch(self, inputs):
        self.network.eval()
        with torch.no_grad():
            outs = _to_list(self._forward([_as_t(x) for x in _to_list(inputs)]))
        return [o.numpy() for o in outs]

    def _update_metrics(self, outs, labels):
        res = []
        for m in self._metrics:
            r = m.compute(*(outs + [_as_t(l) for l in labels]))
            r = m.update(*_to_list(r))
            res.append(r)
        return res

    def _loader(self, data, batch_size, shuffle, drop_last, num_workers):
        if data is None or isinstance(data, _io.DataLoader):
            return data
        return _io.DataLoader(data, batch_size=batch_size, shuffle=shuffle, drop_last=drop_last, num_workers=num_workers)

    def _split(self, batch):
        batch = _to_list(batch)
        n_in = len(_to_list(self._inputs)) if self._inputs is not None else max(1, len(batch) - (1 if self._loss else 0))
        return batch[:n_in], batch[n_in:]

    def fit(self, train_data=None, eval_data=None, batch_size=1, epochs=1, eval_freq=1, log_freq=10, save_dir=None,
            save_freq=1, verbose=2, drop_last=False, shuffle=True, num_workers=0, callbacks=None, accumulate_grad_batches=1,
            num_iters=None):
        train_loader = self._loader(train_data, batch_size, shuffle, drop_last, num_workers)
        eval_loader = self._loader(eval_data, batch_size, False, False, num_workers)
        steps = len(train_loader) if hasattr(train_loader, "__len__") else None
        cbks = config_callbacks(callbacks, model=self, epochs=epochs, steps=steps, log_freq=log_freq,
                                save_freq=save_freq, save_dir=save_dir, verbose=verbose,
                                metrics=["loss"] + [n for m in self._metrics for n in _to_list(m.name())])
        cbks.on_begin("train")
        it = 0
        for epoch in range(epochs):
            cbks.on_epoch_begin(epoch)
            for m in self._metrics:
                m.reset()
            logs = {}
            for step, batch in enumerate(train_loader):
                cbks.on_batch_begin("train", step, logs)
                ins, labs = self._split(batch)
                update = (step + 1) % accumulate_grad_batches == 0
                res = self.train_batch(ins, labs, update=update)
                logs = self._logs(res, step, batch_size)
                cbks.on_batch_end("train", step, logs)
                it += 1
                if num_iters is not None and it >= num_iters:
                    break
            cbks.on_epoch_end(epoch, logs)
            if eval_loader is not None and (epoch + 1) % eval_freq == 0:
                self.evaluate(eval_loader, batch_size=batch_size, verbose=verbose, callbacks=cbks)
            if self.stop_training or (num_iters is not None and it >= num_iters):
                break
        cbks.on_end("train", logs)

    def _logs(self, res, step, batch_size):
        logs = {"step": step, "batch_size": batch_size}
        if isinstance(res, tuple):
            losses, metrics = res
        else:
            losses, metrics = res, []
        if losses:
            logs["loss"] = losses
        for m, r in zip(self._metrics, metrics):
            names = _to_list(m.name())
            vals = _to_list(m.accumulate())
            for n, v in zip(names, vals):
                logs[n] = v
        return logs

    def evaluate(self, eval_data, batch_size=1, log_freq=10, verbose=2, num_workers=0, callbacks=None, num_iters=None):
        loader = self._loader(eval_data, batch_size, False, False, num_workers)
        cbks = callbacks if isinstance(callbacks, cbks_mod.CallbackList) else config_callbacks(callbacks, model=self, verbose=verbose)
        for m in self._metrics:
            m.reset()
        cbks.on_begin("eval")
        logs, losses = {}, []
        for step, batch in enumerate(loader):
            ins, labs = self._split(batch)
            res = self.eval_batch(ins, labs)
            logs = self._logs(res, step, batch_size)
            if "loss" in logs:
                losses.append(logs["loss"])
            cbks.on_batch_end("eval", step, logs)
            if num_iters is not None and step + 1 >= num_iters:
                break
        if losses:
            logs["loss"] = list(np.mean(np.asarray(losses), 0))
        cbks.on_end("eval", logs)
        return {k: v for k, v in logs.items() if k not in ("step", "batch_size")}

    def predict(self, test_data, batch_size=1, num_workers=0, stack_outputs=False, verbose=1, callbacks=None):
        loader = self._loader(test_data, batch_size, False, False, num_workers)
        outs = []
        for batch in loader:
            ins, _ = self._split(batch) if self._inputs is not None else (_to_list(batch)[:1], None)
            outs.append(self.predict_batch(ins))
        res = list(zip(*outs))
        if stack_outputs:
            res = [np.concatenate(r, 0) for r in res]
        return res

    def save(self, path, training=True):
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
        if training:
            _save(self.network.state_dict(), path + ".pdparams")
            if self._optimizer is not None:
                _save(self._optimizer.state_dict(), path + ".pdopt")
        else:
            from .. import jit
            specs = self._inputs if self._inputs is not None else None
            jit.save(self.network, path, input_spec=_to_list(specs))

    def load(self, path, skip_mismatch=False, reset_optimizer=False):
        sd = _load(path + ".pdparams" if not path.endswith(".pdparams") else path)
        self.network.set_state_dict(sd)
        opt_path = (path[:-len(".pdparams")] if path.endswith(".pdparams") else path) + ".pdopt"
        if not reset_optimizer and self._optimizer is not None and os.path.exists(opt_path):
            self._optimizer.set_state_dict(_load(opt_path))

    def parameters(self, *args, **kwargs):
        return self.network.parameters(*args, **kwargs)

    def summary(self, input_size=None, dtype=None):
        return summary(self.network, input_size or [tuple(s.shape) for s in _to_list(self._inputs)], dtype)


def _as_t(x):
    if isinstance(x, Tensor):
        return x
    return to_tensor(np.asarray(x))


def summary(net, input_size=None, dtypes=None, input=None):
    """Per-layer output shapes and parameter counts (reference: hapi/model_summary.py)."""
    rows = []
    hooks = []

    def hook(layer, inputs, out):
        o = out[0] if isinstance(out, (list, tuple)) else out
        n_params = sum(p._t.numel() for p in layer._parameters.values() if p is not None)
        rows.append((f"{type(layer).__name__}-{len(rows) + 1}", list(o.shape) if isinstance(o, Tensor) else None, n_params))

    for l in net.sublayers(include_self=False):
        if not l._sub_layers:
            hooks.append(l.register_forward_post_hook(hook))
    if input is None:
        sizes = input_size if isinstance(input_size, list) and input_size and isinstance(input_size[0], (list, tuple)) else [input_size]
        dts = _to_list(dtypes) or ["float32"] * len(sizes)
        input = [to_tensor(np.zeros([1 if (s is None or s == -1) else s for s in size], dtype=dt)) for size, dt in zip(sizes, dts)]
    was = net.training
    net.eval()
    with torch.no_grad():
        net(*_to_list(input))
    if was:
        net.train()
    for h in hooks:
        h.remove()
    total = sum(p._t.numel() for p in net.parameters())
    trainable = sum(p._t.numel() for p in net.parameters() if p.trainable)
    print("-" * 75)
    print(f"{'Layer (type)':<30}{'Output Shape':<30}{'Param #':>12}")
    print("=" * 75)
    for n, s, p in rows:
        print(f"{n:<30}{str(s):<30}{p:>12,}")
    print("=" * 75)
    print(f"Total params: {total:,}\nTrainable params: {trainable:,}\nNon-trainable params: {total - trainable:,}")
    return {"total_params": total, "trainable_params": trainable}


def flops(net, input_size, custom_ops=None, print_detail=False):
    """Multiply-accumulate count of conv/linear/norm layers via forward hooks (reference: dynamic_flops.py)."""
    from .. import nn
    total = [0]

    def hook(layer, inputs, out):
        o = out[0] if isinstance(out, (list, tuple)) else out
        n_out = int(np.prod(o.shape))
        if custom_ops and type(layer) in custom_ops:
            total[0] += custom_ops[type(layer)](layer, inputs, out)
        elif isinstance(layer, nn.layer.conv_norm_pool._ConvNd):
            k = int(np.prod(layer.weight.shape[1:]))
            total[0] += n_out * k + (n_out if layer.bias is not None else 0)
        elif isinstance(layer, nn.Linear):
            total[0] += n_out * layer.weight.shape[0] + (n_out if layer.bias is not None else 0)
        elif isinstance(layer, (nn.layer.conv_norm_pool._BatchNormBase, nn.LayerNorm)):
            total[0] += 2 * n_out

    hooks = [l.register_forward_post_hook(hook) for l in net.sublayers(include_self=True) if not l._sub_layers]
    x = to_tensor(np.zeros([1 if s in (None, -1) else s for s in input_size], "float32"))
    was = net.training
    net.eval()
    with torch.no_grad():
        net(x)
    if was:
        net.train()
    for h in hooks:
        h.remove()
    if print_detail:
        print(f"Total Flops: {total[0]}")
    return total[0]
