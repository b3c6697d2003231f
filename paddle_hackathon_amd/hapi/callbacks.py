"""Training callbacks (reference: python/paddle/hapi/callbacks.py)."""
from __future__ import annotations

import numbers
import os
import time

import numpy as np

__all__ = ["Callback", "ProgBarLogger", "ModelCheckpoint", "VisualDL", "LRScheduler", "EarlyStopping",
           "ReduceLROnPlateau", "CallbackList", "config_callbacks"]


class Callback:
    def __init__(self):
        self.model = None
        self.params = {}

    def set_params(self, params):
        self.params = params

    def set_model(self, model):
        self.model = model

    def on_train_begin(self, logs=None): pass
    def on_train_end(self, logs=None): pass
    def on_eval_begin(self, logs=None): pass
    def on_eval_end(self, logs=None): pass
    def on_predict_begin(self, logs=None): pass
    def on_predict_end(self, logs=None): pass
    def on_epoch_begin(self, epoch, logs=None): pass
    def on_epoch_end(self, epoch, logs=None): pass
    def on_train_batch_begin(self, step, logs=None): pass
    def on_train_batch_end(self, step, logs=None): pass
    def on_eval_batch_begin(self, step, logs=None): pass
    def on_eval_batch_end(self, step, logs=None): pass
    def on_predict_batch_begin(self, step, logs=None): pass
    def on_predict_batch_end(self, step, logs=None): pass


class CallbackList:
    def __init__(self, callbacks=None):
        self.callbacks = list(callbacks or [])

    def append(self, cb):
        self.callbacks.append(cb)

    def set_model(self, model):
        for c in self.callbacks:
            c.set_model(model)

    def set_params(self, params):
        for c in self.callbacks:
            c.set_params(params)

    def _call(self, name, *args):
        for c in self.callbacks:
            getattr(c, name)(*args)

    def on_begin(self, mode, logs=None):
        self._call(f"on_{mode}_begin", logs)

    def on_end(self, mode, logs=None):
        self._call(f"on_{mode}_end", logs)

    def on_epoch_begin(self, epoch=None, logs=None):
        self._call("on_epoch_begin", epoch, logs)

    def on_epoch_end(self, epoch=None, logs=None):
        self._call("on_epoch_end", epoch, logs)

    def on_batch_begin(self, mode, step=None, logs=None):
        self._call(f"on_{mode}_batch_begin", step, logs)

    def on_batch_end(self, mode, step=None, logs=None):
        self._call(f"on_{mode}_batch_end", step, logs)


class ProgBarLogger(Callback):
    def __init__(self, log_freq=1, verbose=2):
        super().__init__()
        self.log_freq, self.verbose = log_freq, verbose

    def on_epoch_begin(self, epoch, logs=None):
        self.epoch = epoch
        self._t0 = time.time()
        if self.verbose:
            print(f"Epoch {epoch + 1}/{self.params.get('epochs', '?')}")

    def _fmt(self, logs):
        out = []
        for k, v in (logs or {}).items():
            if k in ("step", "batch_size"):
                continue
            if isinstance(v, (list, tuple)):
                v = v[0] if len(v) == 1 else v
            out.append(f"{k}: {v:.4f}" if isinstance(v, numbers.Number) else f"{k}: {v}")
        return " - ".join(out)

    def on_train_batch_end(self, step, logs=None):
        if self.verbose and (step + 1) % self.log_freq == 0:
            print(f"step {step + 1}/{self.params.get('steps', '?')} - {self._fmt(logs)}")

    def on_eval_end(self, logs=None):
        if self.verbose:
            print(f"Eval - {self._fmt(logs)}")


class ModelCheckpoint(Callback):
    def __init__(self, save_freq=1, save_dir=None):
        super().__init__()
        self.save_freq, self.save_dir = save_freq, save_dir

    def on_epoch_end(self, epoch, logs=None):
        if self.save_dir and (epoch + 1) % self.save_freq == 0:
            self.model.save(os.path.join(self.save_dir, str(epoch)))

    def on_train_end(self, logs=None):
        if self.save_dir:
            self.model.save(os.path.join(self.save_dir, "final"))


class VisualDL(Callback):
    """Scalar logger writing JSON lines (VisualDL itself is not available offline)."""

    def __init__(self, log_dir):
        super().__init__()
        self.log_dir = log_dir
        os.makedirs(log_dir, exist_ok=True)
        self._step = 0

    def on_train_batch_end(self, step, logs=None):
        import json
        self._step += 1
        with open(os.path.join(self.log_dir, "scalars.jsonl"), "a") as f:
            f.write(json.dumps({"step": self._step, **{k: (v if isinstance(v, numbers.Number) else np.asarray(v).tolist())
                                                      for k, v in (logs or {}).items()}}) + "\n")


class LRScheduler(Callback):
    def __init__(self, by_step=True, by_epoch=False):
        super().__init__()
        self.by_step, self.by_epoch = by_step, by_epoch

    def _sched(self):
        from ..optimizer.lr import LRScheduler as S
        opt = getattr(self.model, "_optimizer", None)
        lr = getattr(opt, "_learning_rate", None)
        return lr if isinstance(lr, S) else None

    def on_train_batch_end(self, step, logs=None):
        s = self._sched()
        if self.by_step and s is not None:
            s.step()

    def on_epoch_end(self, epoch, logs=None):
        s = self._sched()
        if self.by_epoch and s is not None:
            s.step()


class EarlyStopping(Callback):
    def __init__(self, monitor="loss", mode="auto", patience=0, verbose=1, min_delta=0, baseline=None,
                 save_best_model=True):
        super().__init__()
        self.monitor, self.patience, self.verbose = monitor, patience, verbose
        self.min_delta, self.baseline, self.save_best_model = abs(min_delta), baseline, save_best_model
        if mode == "auto":
            mode = "max" if "acc" in monitor else "min"
        self.op = np.less if mode == "min" else np.greater
        self.min_delta *= -1 if mode == "min" else 1
        self.wait_epoch = 0
        self.best_value = np.inf if mode == "min" else -np.inf
        self.stopped_epoch = 0

    def on_eval_end(self, logs=None):
        if logs is None or self.monitor not in logs:
            return
        cur = logs[self.monitor]
        cur = cur[0] if isinstance(cur, (list, tuple)) else cur
        if self.op(cur - self.min_delta, self.best_value):
            self.best_value = cur
            self.wait_epoch = 0
        else:
            self.wait_epoch += 1
            if self.wait_epoch >= self.patience:
                self.model.stop_training = True


class ReduceLROnPlateau(Callback):
    def __init__(self, monitor="loss", factor=0.1, patience=10, verbose=1, mode="auto", min_delta=1e-4, cooldown=0,
                 min_lr=0):
        super().__init__()
        self.monitor, self.factor, self.patience, self.min_lr = monitor, factor, patience, min_lr
        self.cooldown, self.min_delta = cooldown, min_delta
        self.mode = ("max" if "acc" in monitor else "min") if mode == "auto" else mode
        self.best = np.inf if self.mode == "min" else -np.inf
        self.wait = 0
        self.cooldown_counter = 0

    def on_eval_end(self, logs=None):
        if logs is None or self.monitor not in logs:
            return
        cur = logs[self.monitor]
        cur = cur[0] if isinstance(cur, (list, tuple)) else cur
        better = cur < self.best - self.min_delta if self.mode == "min" else cur > self.best + self.min_delta
        if self.cooldown_counter > 0:
            self.cooldown_counter -= 1
            self.wait = 0
        if better:
            self.best = cur
            self.wait = 0
        elif self.cooldown_counter <= 0:
            self.wait += 1
            if self.wait >= self.patience:
                opt = self.model._optimizer
                old = opt.get_lr()
                if old > self.min_lr:
                    opt.set_lr(max(old * self.factor, self.min_lr))
                self.cooldown_counter = self.cooldown
                self.wait = 0


def config_callbacks(callbacks=None, model=None, batch_size=None, epochs=None, steps=None, log_freq=2, verbose=2,
                     save_freq=1, save_dir=None, metrics=None, mode="train"):
    cbks = list(callbacks or [])
    if not any(isinstance(k, ProgBarLogger) for k in cbks) and verbose:
        cbks = [ProgBarLogger(log_freq, verbose=verbose)] + cbks
    if not any(isinstance(k, ModelCheckpoint) for k in cbks):
        cbks = cbks + [ModelCheckpoint(save_freq, save_dir)]
    if not any(isinstance(k, LRScheduler) for k in cbks):
        cbks = cbks + [LRScheduler()]
    cl = CallbackList(cbks)
    cl.set_model(model)
    cl.set_params({"batch_size": batch_size, "epochs": epochs, "steps": steps, "verbose": verbose, "metrics": metrics or []})
    return cl
