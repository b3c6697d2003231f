"""Dataset trainers: ``Executor.train_from_dataset`` / ``infer_from_dataset`` with device workers
(reference: python/paddle/fluid/executor.py:1773,2396 ``_run_from_dataset``,
fluid/trainer_desc.py:295 MultiTrainer / DistMultiTrainer / PipelineTrainer, fluid/device_worker.py:75
Hogwild, :331 DownpourSGD, :545 Section, fluid/trainer_factory.py:34 TrainerFactory /
FetchHandlerMonitor; C++ paddle/fluid/framework/multi_trainer.cc, hogwild_worker.cc).

A trainer runs ``thread_num`` host worker threads. One reader thread walks the dataset (the
``InMemoryDataset`` / ``QueueDataset`` MultiSlot batches parsed by csrc/runtime/datafeed.cpp) into
a bounded channel; each worker pops batches and interprets the Program on them against the shared
scope (Hogwild: parameters shared, no per-thread copies; forward / backward of the workers run
concurrently and each worker's optimizer step is applied atomically — static/backward.py). In
parameter-server mode (a fleet PS program: its embedding / dense ops pull from and push to the
native table server ``csrc/runtime/ps.cpp``) the workers are DownpourSGD workers: the same loop,
the pulls and pushes being part of the program. Worker 0 prints the ``fetch_list`` values with
their ``fetch_info`` labels every ``print_period`` batches; a ``FetchHandler`` is polled from a
monitor thread every ``period_secs`` with the named variables' values from the scope."""
from __future__ import annotations

import queue
import sys
import threading
import time

import numpy as np

__all__ = ["DeviceWorker", "Hogwild", "DownpourSGD", "DownpourSGDOPT", "Section", "HeterSection",
           "TrainerDesc", "MultiTrainer", "DistMultiTrainer", "HeterXpuTrainer", "PSGPUTrainer", "HeterPipelineTrainer",
           "PipelineTrainer", "TrainerFactory", "FetchHandler", "FetchHandlerMonitor"]


# ---------------------------------------------------------------------------------- hogwild sync
class _RWLock:
    """writer-preferring read / write lock: a worker's forward + backward hold the read side (many
    at once), its optimizer step the write side — in-place parameter updates never land inside
    another worker's forward / backward (torch's saved-tensor version checks would reject the
    gradient), and a waiting update keeps new batches from starting until it has been applied"""

    def __init__(self):
        self._c = threading.Condition()
        self._readers = 0
        self._writer = False
        self._waiting = 0

    def acquire_read(self):
        with self._c:
            while self._writer or self._waiting:
                self._c.wait()
            self._readers += 1

    def release_read(self):
        with self._c:
            self._readers -= 1
            if not self._readers:
                self._c.notify_all()

    def acquire_write(self):
        with self._c:
            self._waiting += 1
            while self._writer or self._readers:
                self._c.wait()
            self._waiting -= 1
            self._writer = True

    def release_write(self):
        with self._c:
            self._writer = False
            self._c.notify_all()


class _Worker(threading.local):
    def __init__(self):
        self.rw = None          # the trainer's lock while this thread is a worker
        self.reading = False    # holds the read side (inside a batch, before its update)
        self.alias = False      # lock-free Hogwild: the batch reads parameter aliases (see below)


def hogwild_alias():
    """inside a lock-free Hogwild worker: run_program binds every trainable parameter to an alias
    sharing its storage with its own autograd version counter (``tensor.data``), so other threads'
    in-place updates land in this batch's reads (Hogwild's racy reads) without invalidating the
    tensors its backward saved; the update is applied to the real parameter"""
    return _WORKER.alias


_WORKER = _Worker()


class hogwild_update:
    """context of an optimizer op: inside a dataset-trainer worker, trade the batch's read lock for
    the write lock for the update (static/backward.py)"""

    def __enter__(self):
        w = _WORKER
        self._rw = w.rw
        if self._rw is not None:
            if w.reading:
                self._rw.release_read()
                w.reading = False
            self._rw.acquire_write()
        return self

    def __exit__(self, *exc):
        if self._rw is not None:
            self._rw.release_write()
        return False


# ---------------------------------------------------------------------------------- device workers
class DeviceWorker:
    """what one trainer thread runs per batch (device_worker.py:24)"""

    def __init__(self):
        self._program = None
        self._infer = False
        self._fleet_desc = None

    def _set_infer(self, infer=False):
        self._infer = infer

    def _set_fleet_desc(self, fleet_desc):
        self._fleet_desc = fleet_desc

    def _set_program(self, program):
        self._program = program

    def _gen_worker_desc(self, trainer_desc):
        trainer_desc.device_worker_name = type(self).__name__ + "Worker"

    def run_batch(self, executor, program, batch, fetch_list, scope):
        from .program import run_program
        return run_program(program, batch, fetch_list, scope)


class Hogwild(DeviceWorker):
    """lock-free asynchronous SGD over shared parameters (hogwild_worker.cc: every thread runs the
    whole program on its batches against the shared parameters; no thread waits for another's
    forward / backward). Each batch reads parameter aliases (``hogwild_alias``): other threads'
    updates show up in its reads while it runs, as in the reference, and its own update is one
    optimizer step on the real parameters, serialised only against other updates (the
    optimizer's state is one object)"""
    lock_free = True


class DownpourSGD(Hogwild):
    """parameter-server worker (downpour_worker.cc): Hogwild threads whose program pulls its
    sparse rows / dense tables before the batch and pushes their gradients after it (the fleet PS
    program's own pull / push ops, parallel/ps); the server applies pushes asynchronously"""


class DownpourSGDOPT(DownpourSGD):
    """downpour_worker_opt.cc: the same loop (the reference variant differs in its C++ scheduling
    of pulls only)"""


class Section(DeviceWorker):
    """pipeline section worker (section_worker.cc): the program is a pipeline stage driven by the
    static pipeline runner (parallel/fleet/static_pipeline.py) over micro-batches"""

    def run_batch(self, executor, program, batch, fetch_list, scope):
        pipe = program.__dict__.get("_pipeline")
        if pipe is not None:
            return pipe.run(batch, fetch_list or [])
        return super().run_batch(executor, program, batch, fetch_list, scope)


class HeterSection(Section):
    pass


# ---------------------------------------------------------------------------------- trainers
class TrainerDesc:
    """the trainer configuration (trainer_desc.py:27; the reference serialises it to a protobuf
    for the C++ trainer — here the Python trainer reads it directly)"""

    def __init__(self):
        self.thread_num = 1
        self.device_worker = None
        self.fetch_vars, self.fetch_info, self.print_period = [], [], 100
        self.debug = False
        self.infer = False
        self.scope = None
        self.device_worker_name = ""
        self.dump_fields, self.dump_fields_path = [], None

    def _set_thread(self, thread_num):
        self.thread_num = max(1, int(thread_num))

    def _set_device_worker(self, device_worker):
        self.device_worker = device_worker

    def _set_infer(self, infer):
        self.infer = infer
        if self.device_worker is not None:
            self.device_worker._set_infer(infer)

    def _set_fetch_var_and_info(self, fetch_vars, fetch_info, print_period):
        self.fetch_vars, self.fetch_info, self.print_period = list(fetch_vars or []), list(fetch_info or []), \
            int(print_period)

    def _set_debug(self, debug):
        self.debug = bool(debug)

    def _set_program(self, program):
        self._program = program

    def _set_dump_fields(self, fields, path=None):
        self.dump_fields, self.dump_fields_path = list(fields or []), path

    def _desc(self):
        return (f"{type(self).__name__}(thread_num={self.thread_num}, device_worker="
                f"{type(self.device_worker).__name__ if self.device_worker else None})")

    def run(self, executor, program, dataset, scope, fetch_handler=None):
        return _run_trainer(self, executor, program, dataset, scope, fetch_handler)


class MultiTrainer(TrainerDesc):
    pass


class DistMultiTrainer(TrainerDesc):
    pass


class HeterXpuTrainer(TrainerDesc):
    pass


class PSGPUTrainer(TrainerDesc):
    pass


class HeterPipelineTrainer(TrainerDesc):
    pass


class PipelineTrainer(TrainerDesc):
    pass


def _is_ps_program(program):
    """a fleet parameter-server program: its ops talk to the table server"""
    return bool(program.__dict__.get("_ps_mode") or program.__dict__.get("_transpiled")
                or any("pull" in op.type or "push" in op.type or op.type in ("send", "recv", "distributed_lookup_table")
                       for b in program.blocks for op in b.ops))


class TrainerFactory:
    """trainer_factory.py:34 — MultiTrainer + Hogwild by default, DistMultiTrainer + DownpourSGD
    for parameter-server programs, PipelineTrainer + Section for static pipelines"""

    def _create_trainer(self, opt_info=None, program=None):
        opt_info = opt_info or {}
        name = opt_info.get("trainer")
        worker = opt_info.get("device_worker")
        if name is None and program is not None:
            if program.__dict__.get("_pipeline") is not None:
                name, worker = "PipelineTrainer", "Section"
            elif _is_ps_program(program):
                name, worker = "DistMultiTrainer", "DownpourSGD"
        trainer = globals()[name or "MultiTrainer"]()
        trainer._set_device_worker(globals()[worker or "Hogwild"]())
        return trainer


# ---------------------------------------------------------------------------------- fetch handler
class FetchHandler:
    """executor.py:502 — ``handler(res_dict)`` is called every ``period_secs`` with the current
    values (numpy) of ``var_dict``'s variables"""

    def __init__(self, var_dict=None, period_secs=60):
        assert var_dict is not None
        self.var_dict = var_dict
        self.period_secs = period_secs

    def handler(self, res_dict):
        for key in res_dict:
            if type(res_dict[key]) is np.ndarray:
                sys.stdout.write("{}[0]: {} ".format(key, res_dict[key][0]))
        sys.stdout.write("\n")

    @staticmethod
    def help():
        print("subclass FetchHandler and override handler(self, res_dict); var_dict = {key: Variable or name}")


class FetchHandlerMonitor:
    """polls the scope every ``period_secs`` (trainer_factory.py:126)"""

    def __init__(self, scope, handler, latest=None):
        self.handler, self.scope, self.latest = handler, scope, latest if latest is not None else {}
        self._stop = threading.Event()
        self.thread = threading.Thread(target=self._loop, daemon=True)

    def start(self):
        self.thread.start()

    def stop(self):
        self._stop.set()
        self.thread.join()

    def _values(self):
        res = {}
        for key, var in self.handler.var_dict.items():
            name = var if isinstance(var, str) else getattr(var, "name", None)
            v = self.latest.get(name)
            if v is None and self.scope is not None and name:
                sv = self.scope.find_var(name)
                v = np.array(sv.get_tensor()) if sv is not None and sv.value is not None else None
            res[key] = v
        return res

    def _loop(self):
        period = max(float(self.handler.period_secs), 0.01)
        last = time.time()
        while not self._stop.wait(0.01):
            if time.time() - last >= period:
                last = time.time()
                self.handler.handler(self._values())
        self.handler.handler(self._values())   # once more at the end of the pass


# ---------------------------------------------------------------------------------- the loop
_END = object()


def _name(v):
    return v if isinstance(v, str) else getattr(v, "name", None) or f"fetch_{id(v)}"


def _run_trainer(trainer, executor, program, dataset, scope, fetch_handler):
    from .program import global_scope, Variable
    scope = scope if scope is not None else global_scope()
    prog = program
    if trainer.infer:
        prog = program.clone(for_test=True)
    fetch_vars = trainer.fetch_vars
    fetch_info = trainer.fetch_info or [_name(v) for v in fetch_vars]
    latest = {}
    chan = queue.Queue(maxsize=max(4, 2 * trainer.thread_num))
    errors = []
    stats = {"batches": [0] * trainer.thread_num, "t0": time.time()}

    def reader():
        try:
            for batch in dataset:
                chan.put(batch)
        except BaseException as e:   # noqa: BLE001 - surfaced by the main thread
            errors.append(e)
        finally:
            for _ in range(trainer.thread_num):
                chan.put(_END)

    rw = _RWLock()

    # Hogwild / Downpour workers on the root scope run lock-free on parameter aliases; other
    # workers (and non-root scopes, whose parameters are the scope's copies) keep the read / write
    # lock between batches and updates
    lock_free = bool(getattr(trainer.device_worker, "lock_free", False)) and not trainer.infer and \
        getattr(scope, "_root", True)

    def worker(tid):
        dw = trainer.device_worker
        _WORKER.rw = None if lock_free else rw
        _WORKER.alias = lock_free
        try:
            while True:
                batch = chan.get()
                if batch is _END:
                    return
                if lock_free:
                    out = dw.run_batch(executor, prog, batch, fetch_vars, scope)
                else:
                    rw.acquire_read()
                    _WORKER.reading = True
                    try:
                        out = dw.run_batch(executor, prog, batch, fetch_vars, scope)
                    finally:
                        if _WORKER.reading:
                            _WORKER.reading = False
                            rw.release_read()
                stats["batches"][tid] += 1
                if fetch_vars and out:
                    vals = [o.numpy() if hasattr(o, "numpy") else np.asarray(o) for o in out]
                    for v, val in zip(fetch_vars, vals):
                        latest[_name(v)] = val
                    if tid == 0 and trainer.print_period > 0 and stats["batches"][0] % trainer.print_period == 0:
                        print(" ".join(f"{info}: {np.asarray(val).reshape(-1)[:8].tolist()}"
                                       for info, val in zip(fetch_info, vals)), flush=True)
        except BaseException as e:   # noqa: BLE001 - surfaced by the main thread
            errors.append(e)
            while chan.get() is not _END:   # drain so the reader can finish
                pass
        finally:
            _WORKER.rw = None
            _WORKER.alias = False

    mon = FetchHandlerMonitor(scope, fetch_handler, latest) if fetch_handler is not None else None
    if mon is not None:
        mon.start()
    rt = threading.Thread(target=reader, daemon=True)
    rt.start()
    ws = [threading.Thread(target=worker, args=(i,), daemon=True) for i in range(trainer.thread_num)]
    for w in ws:
        w.start()
    for w in ws:
        w.join()
    rt.join()
    if mon is not None:
        mon.stop()
    if errors:
        raise errors[0]
    if trainer.debug:
        dt = time.time() - stats["t0"]
        print(f"[{type(trainer).__name__}] {sum(stats['batches'])} batches in {dt:.3f}s over "
              f"{trainer.thread_num} threads: {stats['batches']}", flush=True)
    _ = Variable
    return None


def run_from_dataset(executor, program, dataset, scope, thread, is_infer, debug, fetch_list, fetch_info,
                     print_period, fetch_handler):
    """executor.py:1773 _run_from_dataset"""
    from .program import default_main_program
    if dataset is None:
        raise RuntimeError("dataset is needed and should be initialized")
    program = program if program is not None else default_main_program()
    opt_info = program.__dict__.get("_fleet_opt")
    trainer = TrainerFactory()._create_trainer(opt_info, program)
    trainer._set_thread(thread if thread and thread > 0 else getattr(dataset, "thread_num", 1))
    trainer._set_infer(is_infer)
    trainer._set_debug(debug)
    trainer._set_fetch_var_and_info(fetch_list, fetch_info, print_period)
    trainer._set_program(program)
    return trainer.run(executor, program, dataset, scope, fetch_handler)
