"""Auto-checkpoint / resume (reference: python/paddle/fluid/incubate/checkpoint/
auto_checkpoint.py, exposed as paddle.incubate.checkpoint).

``for epoch in train_epoch_range(N): ...`` resumes from the last completed epoch found in
the checkpoint directory and, after each epoch (every ``save_checkpoint_inter`` seconds at
most), saves every registered Layer / Optimizer state of this rank. Saves are atomic
(write to a temp dir, then rename), so a rank killed mid-save never leaves a torn
checkpoint; the newest ``keep`` checkpoints are kept.

Environment (same names as the reference where they exist):
  PADDLE_RUNNING_ENV=PADDLE_EDL_AUTO_CHECKPOINT  enables it (or pass ``enable=True``)
  PADDLE_EDL_HDFS_CHECKPOINT_PATH / PHA_CHECKPOINT_DIR   checkpoint root
  PADDLE_JOB_ID                                   job namespace (default "default")
"""
from __future__ import annotations

import json
import os
import shutil
import time

from ...framework.io import save as _save, load as _load

__all__ = ["train_epoch_range", "register", "AutoCheckpointChecker", "latest_checkpoint"]

_registry = {}


def register(**objs):
    """register(model=layer, opt=optimizer, ...): objects with state_dict/set_state_dict."""
    _registry.update(objs)


class AutoCheckpointChecker:
    def __init__(self, enable=None, root=None, job_id=None):
        env = os.environ
        self.run_env = env.get("PADDLE_RUNNING_ENV", "")
        self.enabled = (self.run_env == "PADDLE_EDL_AUTO_CHECKPOINT") if enable is None else enable
        self.root = root or env.get("PHA_CHECKPOINT_DIR") or env.get("PADDLE_EDL_HDFS_CHECKPOINT_PATH") or "./auto_checkpoint"
        self.job_id = job_id or env.get("PADDLE_JOB_ID", "default")
        self.rank = int(env.get("PADDLE_TRAINER_ID", env.get("RANK", "0")))
        self.save_inter = int(env.get("PADDLE_EDL_SAVE_CHECKPOINT_INTER", "900"))

    @property
    def job_dir(self):
        return os.path.join(self.root, self.job_id)


def _epochs(job_dir):
    if not os.path.isdir(job_dir):
        return []
    out = []
    for d in os.listdir(job_dir):
        if d.startswith("epoch_") and os.path.exists(os.path.join(job_dir, d, "meta.json")):
            try:
                out.append(int(d[len("epoch_"):]))
            except ValueError:
                pass
    return sorted(out)


def latest_checkpoint(checker=None):
    c = checker or AutoCheckpointChecker(enable=True)
    e = _epochs(c.job_dir)
    return (e[-1], os.path.join(c.job_dir, f"epoch_{e[-1]}")) if e else (None, None)


def _save_epoch(c, epoch, keep):
    final = os.path.join(c.job_dir, f"epoch_{epoch}")
    tmp = final + f".tmp.{c.rank}.{os.getpid()}"
    os.makedirs(tmp, exist_ok=True)
    for name, obj in _registry.items():
        _save(obj.state_dict(), os.path.join(tmp, f"{name}.rank{c.rank}.pdstate"))
    os.makedirs(final, exist_ok=True)
    for f in os.listdir(tmp):
        os.replace(os.path.join(tmp, f), os.path.join(final, f))
    shutil.rmtree(tmp, ignore_errors=True)
    if c.rank == 0:
        with open(os.path.join(final, "meta.json.tmp"), "w") as fh:
            json.dump({"epoch": epoch, "time": time.time(), "objects": sorted(_registry)}, fh)
        os.replace(os.path.join(final, "meta.json.tmp"), os.path.join(final, "meta.json"))
        for old in _epochs(c.job_dir)[:-keep]:
            shutil.rmtree(os.path.join(c.job_dir, f"epoch_{old}"), ignore_errors=True)


def _restore(path, c):
    for name, obj in _registry.items():
        f = os.path.join(path, f"{name}.rank{c.rank}.pdstate")
        if os.path.exists(f):
            obj.set_state_dict(_load(f))


def train_epoch_range(max_epoch_num, save_checkpoint_inter=None, enable=None, keep=2):
    c = AutoCheckpointChecker(enable=enable)
    if not c.enabled:
        yield from range(max_epoch_num)
        return
    inter = c.save_inter if save_checkpoint_inter is None else save_checkpoint_inter
    last, path = latest_checkpoint(c)
    start = 0
    if last is not None:
        _restore(path, c)
        start = last + 1
    t_last = time.time()
    for epoch in range(start, max_epoch_num):
        yield epoch
        if time.time() - t_last >= inter or epoch == max_epoch_num - 1:
            _save_epoch(c, epoch, keep)
            t_last = time.time()
