"""``paddle.io`` data pipeline (reference: python/paddle/fluid/dataloader/*,
python/paddle/fluid/reader.py, paddle/fluid/imperative/data_loader.cc).

DataLoader = sampler → (optional) worker processes → collate → buffered reader.
The buffered reader stages host batches in pinned memory and copies them to the
HIP device on a side stream one batch ahead (``use_buffer_reader``), so H2D
copies overlap the previous step's compute. Collation of numpy samples goes
through the native C++ collator when the runtime library is built
(csrc/runtime/collate.cpp), else numpy.
"""
from __future__ import annotations

import itertools
import math
import multiprocessing as mp
import queue
import os
import threading

import numpy as np
import torch

from ..framework.core import Tensor, _wrap, default_device

__all__ = ["Dataset", "IterableDataset", "TensorDataset", "ComposeDataset", "ChainDataset", "Subset", "random_split",
           "Sampler", "SequenceSampler", "RandomSampler", "WeightedRandomSampler", "BatchSampler",
           "DistributedBatchSampler", "DataLoader", "get_worker_info", "default_collate_fn"]


class Dataset:
    def __getitem__(self, idx):
        raise NotImplementedError

    def __len__(self):
        raise NotImplementedError


class IterableDataset(Dataset):
    def __iter__(self):
        raise NotImplementedError

    def __getitem__(self, idx):
        raise RuntimeError("IterableDataset does not support indexing")

    def __len__(self):
        raise RuntimeError("IterableDataset has no len()")


class TensorDataset(Dataset):
    def __init__(self, tensors):
        n = tensors[0].shape[0]
        assert all(t.shape[0] == n for t in tensors)
        self.tensors = tensors

    def __getitem__(self, index):
        return tuple(t[index] for t in self.tensors)

    def __len__(self):
        return self.tensors[0].shape[0]


class ComposeDataset(Dataset):
    def __init__(self, datasets):
        self.datasets = list(datasets)

    def __len__(self):
        return len(self.datasets[0])

    def __getitem__(self, idx):
        out = []
        for d in self.datasets:
            s = d[idx]
            out.extend(s if isinstance(s, (list, tuple)) else [s])
        return tuple(out)


class ChainDataset(IterableDataset):
    def __init__(self, datasets):
        self.datasets = list(datasets)

    def __iter__(self):
        for d in self.datasets:
            yield from d


class Subset(Dataset):
    def __init__(self, dataset, indices):
        self.dataset, self.indices = dataset, list(indices)

    def __getitem__(self, idx):
        return self.dataset[self.indices[idx]]

    def __len__(self):
        return len(self.indices)


def random_split(dataset, lengths, generator=None):
    n = len(dataset)
    if all(0 < l < 1 for l in lengths) and abs(sum(lengths) - 1) < 1e-6:
        lengths = [int(math.floor(n * f)) for f in lengths]
        for i in range(n - sum(lengths)):
            lengths[i % len(lengths)] += 1
    assert sum(lengths) == n
    perm = np.random.permutation(n).tolist()
    out, off = [], 0
    for l in lengths:
        out.append(Subset(dataset, perm[off:off + l]))
        off += l
    return out


class Sampler:
    def __init__(self, data_source=None):
        self.data_source = data_source

    def __iter__(self):
        raise NotImplementedError


class SequenceSampler(Sampler):
    def __iter__(self):
        return iter(range(len(self.data_source)))

    def __len__(self):
        return len(self.data_source)


class RandomSampler(Sampler):
    def __init__(self, data_source, replacement=False, num_samples=None, generator=None):
        super().__init__(data_source)
        self.replacement, self._num_samples, self.generator = replacement, num_samples, generator

    @property
    def num_samples(self):
        return len(self.data_source) if self._num_samples is None else self._num_samples

    def __iter__(self):
        n = len(self.data_source)
        if self.generator is not None:
            yield from (next(self.generator) for _ in range(self.num_samples))
            return
        if self.replacement:
            yield from np.random.randint(0, n, self.num_samples).tolist()
        else:
            yield from np.random.permutation(n).tolist()[: self.num_samples]

    def __len__(self):
        return self.num_samples


class WeightedRandomSampler(Sampler):
    def __init__(self, weights, num_samples, replacement=True):
        super().__init__()
        w = np.asarray(weights._t.cpu().numpy() if isinstance(weights, Tensor) else weights, dtype=np.float64)
        self.weights = w / w.sum()
        self.num_samples, self.replacement = num_samples, replacement

    def __iter__(self):
        yield from np.random.choice(len(self.weights), self.num_samples, self.replacement, self.weights).tolist()

    def __len__(self):
        return self.num_samples


class BatchSampler(Sampler):
    def __init__(self, dataset=None, sampler=None, shuffle=False, batch_size=1, drop_last=False):
        if sampler is None:
            sampler = RandomSampler(dataset) if shuffle else SequenceSampler(dataset)
        self.sampler, self.batch_size, self.drop_last = sampler, batch_size, drop_last

    def __iter__(self):
        batch = []
        for i in self.sampler:
            batch.append(i)
            if len(batch) == self.batch_size:
                yield batch
                batch = []
        if batch and not self.drop_last:
            yield batch

    def __len__(self):
        n = len(self.sampler)
        return n // self.batch_size if self.drop_last else (n + self.batch_size - 1) // self.batch_size


class DistributedBatchSampler(BatchSampler):
    """Each rank sees a disjoint 1/nranks slice (padded to equal length), reshuffled per epoch."""

    def __init__(self, dataset, batch_size, num_replicas=None, rank=None, shuffle=False, drop_last=False):
        self.dataset, self.batch_size, self.shuffle, self.drop_last = dataset, batch_size, shuffle, drop_last
        if num_replicas is None or rank is None:
            from ..parallel.collective import get_rank, get_world_size
            num_replicas = get_world_size() if num_replicas is None else num_replicas
            rank = get_rank() if rank is None else rank
        self.nranks, self.local_rank = num_replicas, rank
        self.epoch = 0
        self.num_samples = int(math.ceil(len(dataset) * 1.0 / self.nranks))
        self.total_size = self.num_samples * self.nranks

    def __iter__(self):
        n = len(self.dataset)
        indices = np.arange(n).tolist()
        indices += indices[: (self.total_size - len(indices))]
        if self.shuffle:
            np.random.RandomState(self.epoch).shuffle(indices)
            self.epoch += 1
        # contiguous block per rank, as the reference does
        indices = indices[self.local_rank * self.num_samples:(self.local_rank + 1) * self.num_samples]
        batch = []
        for i in indices:
            batch.append(i)
            if len(batch) == self.batch_size:
                yield batch
                batch = []
        if batch and not self.drop_last:
            yield batch

    def __len__(self):
        n = self.num_samples
        return n // self.batch_size if self.drop_last else (n + self.batch_size - 1) // self.batch_size

    def set_epoch(self, epoch):
        self.epoch = epoch


# ----------------------------------------------------------------------------- collation
def _native_stack(arrs):
    from ..utils import native
    return native.stack_arrays(arrs)


def default_collate_fn(batch):
    sample = batch[0]
    if isinstance(sample, np.ndarray):
        try:
            return _native_stack(batch)
        except Exception:
            return np.stack(batch)
    if isinstance(sample, Tensor):
        return _wrap(torch.stack([b._t for b in batch]))
    if isinstance(sample, torch.Tensor):
        return torch.stack(batch)
    if isinstance(sample, (int, np.integer)):
        return np.asarray(batch, dtype=np.int64)
    if isinstance(sample, (float, np.floating)):
        return np.asarray(batch, dtype=np.float32)
    if isinstance(sample, (str, bytes)):
        return list(batch)
    if isinstance(sample, dict):
        return {k: default_collate_fn([b[k] for b in batch]) for k in sample}
    if isinstance(sample, (list, tuple)):
        return [default_collate_fn(list(f)) for f in zip(*batch)]
    return batch


def default_convert_fn(batch):
    return batch


_worker_info = threading.local()


class _WorkerInfo:
    def __init__(self, id, num_workers, dataset, seed):
        self.id, self.num_workers, self.dataset, self.seed = id, num_workers, dataset, seed


def get_worker_info():
    return getattr(_worker_info, "info", None)


_RING = "__pha_ring__"


def _ring_put(ring, idx, data):
    """Write a collated batch into a free shared-memory slot; False if it does not fit."""
    from ..utils import native
    while True:
        slot = ring.acquire_write(timeout_ms=1000)
        if slot == -2:
            return True  # ring closed: trainer is shutting down
        if slot >= 0:
            break
        if os.getppid() == 1:  # trainer died
            return True
    n = native.pack_into(data, ring.slot_view(slot))
    if n < 0:
        ring.abort(slot)
        return False
    ring.commit(slot, idx, n)
    return True


def _worker_loop(dataset, index_q, out_q, collate_fn, worker_id, num_workers, init_fn, seed, iterable, batch_size,
                 drop_last, ring=None):
    _worker_info.info = _WorkerInfo(worker_id, num_workers, dataset, seed)
    np.random.seed((seed + worker_id) % (2 ** 32))
    torch.manual_seed(seed + worker_id)
    if init_fn is not None:
        init_fn(worker_id)
    if iterable:
        it = iter(dataset)
        batch = []
        for s in it:
            batch.append(s)
            if len(batch) == batch_size:
                out_q.put((None, collate_fn(batch)))
                batch = []
        if batch and not drop_last:
            out_q.put((None, collate_fn(batch)))
        out_q.put((None, StopIteration))
        return
    while True:
        item = index_q.get()
        if item is None:
            break
        idx, indices = item
        try:
            data = collate_fn([dataset[i] for i in indices])
        except Exception as e:  # propagate worker errors
            out_q.put((idx, RuntimeError(f"DataLoader worker {worker_id} failed: {e!r}")))
            continue
        if ring is not None and _is_array_tree(data) and _ring_put(ring, idx, data):
            out_q.put((idx, _RING))
        else:
            out_q.put((idx, data))


def _is_array_tree(x):
    if isinstance(x, np.ndarray):
        return x.dtype != object
    if isinstance(x, dict):
        return all(_is_array_tree(v) for v in x.values())
    if isinstance(x, (list, tuple)):
        return all(_is_array_tree(v) for v in x)
    return isinstance(x, (int, float, str, bytes, np.generic)) or x is None


def _tree_nbytes(x):
    if isinstance(x, np.ndarray):
        return x.nbytes + 64
    if isinstance(x, dict):
        return sum(_tree_nbytes(v) for v in x.values())
    if isinstance(x, (list, tuple)):
        return sum(_tree_nbytes(v) for v in x)
    return 64


def _ring_take(ring, idx, pin):
    """Read batch ``idx`` out of the ring into private (pinned, when feeding a GPU) memory."""
    from ..utils import native
    slot = ring.acquire_read(idx, timeout_ms=60000)
    if slot < 0:
        raise RuntimeError(f"DataLoader shared-memory ring lost batch {idx}")
    try:
        views = native.unpack_from(ring.slot_view(slot, ring.nbytes(slot)), copy=False)

        def own(x):
            if isinstance(x, np.ndarray):
                if pin:
                    t = torch.empty(x.shape, dtype=torch.from_numpy(x[:0].copy()).dtype, pin_memory=True)
                    t.copy_(torch.from_numpy(x))
                    return t
                return x.copy()
            if isinstance(x, dict):
                return {k: own(v) for k, v in x.items()}
            if isinstance(x, (list, tuple)):
                return [own(v) for v in x]
            return x
        return own(views)
    finally:
        ring.release(slot)


def _to_device_tree(x, dev, non_blocking):
    if isinstance(x, np.ndarray):
        t = torch.from_numpy(x)
        if dev.type == "cuda":
            t = t.pin_memory().to(dev, non_blocking=non_blocking)
        return _wrap(t)
    if isinstance(x, Tensor):
        return _wrap(x._t.to(dev, non_blocking=non_blocking))
    if isinstance(x, torch.Tensor):
        return _wrap(x.to(dev, non_blocking=non_blocking))
    if isinstance(x, dict):
        return {k: _to_device_tree(v, dev, non_blocking) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_to_device_tree(v, dev, non_blocking) for v in x]
    return x


def _record_stream_tree(x, stream):
    if isinstance(x, Tensor):
        if x._t.is_cuda:
            x._t.record_stream(stream)
    elif isinstance(x, dict):
        for v in x.values():
            _record_stream_tree(v, stream)
    elif isinstance(x, (list, tuple)):
        for v in x:
            _record_stream_tree(v, stream)


class DataLoader:
    def __init__(self, dataset, feed_list=None, places=None, return_list=True, batch_sampler=None, batch_size=1,
                 shuffle=False, drop_last=False, collate_fn=None, num_workers=0, use_buffer_reader=True,
                 use_shared_memory=True, timeout=0, worker_init_fn=None, persistent_workers=False, prefetch_factor=2):
        self.dataset = dataset
        self.return_list = return_list
        self.num_workers = num_workers
        self.use_buffer_reader = use_buffer_reader
        self.use_shared_memory = use_shared_memory
        self.worker_init_fn = worker_init_fn
        self.timeout = timeout
        self.prefetch_factor = max(2, prefetch_factor)
        self._iterable = isinstance(dataset, IterableDataset)
        self.batch_size = batch_size
        self.drop_last = drop_last
        if self._iterable:
            self.batch_sampler = None
        elif batch_sampler is not None:
            self.batch_sampler = batch_sampler
        elif batch_size is None:
            self.batch_sampler = None
        else:
            self.batch_sampler = BatchSampler(dataset, shuffle=shuffle, batch_size=batch_size, drop_last=drop_last)
        self.collate_fn = collate_fn or (default_collate_fn if batch_size is not None or batch_sampler is not None else default_convert_fn)
        if places is not None:
            from ..framework.core import _to_torch_device
            pl = places[0] if isinstance(places, (list, tuple)) else places
            self.device = _to_torch_device(pl)
        else:
            self.device = default_device()

    def __len__(self):
        if self._iterable:
            raise TypeError("IterableDataset DataLoader has no len()")
        return len(self.batch_sampler) if self.batch_sampler is not None else len(self.dataset)

    def _host_batches(self):
        if self.num_workers == 0:
            if self._iterable:
                batch = []
                for s in self.dataset:
                    if self.batch_size is None:
                        yield self.collate_fn(s)
                        continue
                    batch.append(s)
                    if len(batch) == self.batch_size:
                        yield self.collate_fn(batch)
                        batch = []
                if batch and not self.drop_last:
                    yield self.collate_fn(batch)
                return
            if self.batch_sampler is None:
                for i in range(len(self.dataset)):
                    yield self.collate_fn(self.dataset[i])
                return
            for indices in self.batch_sampler:
                yield self.collate_fn([self.dataset[i] for i in indices])
            return
        yield from self._mp_batches()

    def _mp_batches(self):
        ctx = mp.get_context("fork")
        out_q = ctx.Queue(maxsize=self.num_workers * self.prefetch_factor)
        seed = int(np.random.randint(0, 2 ** 31))
        if self._iterable:
            workers = [ctx.Process(target=_worker_loop, args=(self.dataset, None, out_q, self.collate_fn, w, self.num_workers,
                                                             self.worker_init_fn, seed, True, self.batch_size, self.drop_last),
                                   daemon=True) for w in range(self.num_workers)]
            for p in workers:
                p.start()
            done = 0
            try:
                while done < self.num_workers:
                    _, data = out_q.get(timeout=self.timeout or None)
                    if data is StopIteration:
                        done += 1
                        continue
                    yield data
            finally:
                for p in workers:
                    p.join(timeout=1)
                    if p.is_alive():
                        p.terminate()
            return
        index_qs = [ctx.Queue() for _ in range(self.num_workers)]
        batches = iter(self.batch_sampler)
        first = next(batches, None)
        if first is None:
            return
        ring = self._make_ring(first)
        pin = ring is not None and self.device.type == "cuda"
        workers = [ctx.Process(target=_worker_loop, args=(self.dataset, index_qs[w], out_q, self.collate_fn, w,
                                                         self.num_workers, self.worker_init_fn, seed, False, None,
                                                         False, ring), daemon=True)
                   for w in range(self.num_workers)]
        for p in workers:
            p.start()
        cap = self.num_workers * self.prefetch_factor  # == ring slots: every in-flight batch has a slot
        try:
            sent = 0
            b = first
            while b is not None:
                index_qs[sent % self.num_workers].put((sent, b))
                sent += 1
                b = next(batches, None) if sent < cap else None
            pending = {}
            nxt = 0
            while nxt < sent:
                while nxt not in pending:
                    idx, data = self._get(out_q, workers)
                    if isinstance(data, str) and data == _RING:
                        data = _ring_take(ring, idx, pin)
                    pending[idx] = data
                data = pending.pop(nxt)
                nxt += 1
                b = next(batches, None)
                if b is not None:
                    index_qs[sent % self.num_workers].put((sent, b))
                    sent += 1
                if isinstance(data, Exception):
                    raise data
                yield data
        finally:
            if ring is not None:
                ring.close()
            for q in index_qs:
                q.put(None)
            for p in workers:
                p.join(timeout=1)
                if p.is_alive():
                    p.terminate()
            if ring is not None:
                ring.destroy()

    def _get(self, out_q, workers):
        """out_q.get with a liveness watchdog: a dead worker raises instead of hanging."""
        import queue as _queue
        waited = 0.0
        while True:
            try:
                return out_q.get(timeout=5.0)
            except _queue.Empty:
                waited += 5.0
                dead = [p for p in workers if not p.is_alive() and p.exitcode not in (0, None)]
                if dead:
                    raise RuntimeError(f"DataLoader worker (pid {dead[0].pid}) exited unexpectedly "
                                       f"with code {dead[0].exitcode}")
                if self.timeout and waited >= self.timeout:
                    raise RuntimeError(f"DataLoader timed out after {self.timeout}s")

    def _make_ring(self, first_indices):
        """Shared-memory batch ring sized from one probe batch (None: pickle through the queue)."""
        if not self.use_shared_memory:
            return None
        from ..utils import native
        if not native.available():
            return None
        try:
            probe = self.collate_fn([self.dataset[i] for i in first_indices])
        except Exception:
            return None
        if not _is_array_tree(probe):
            return None
        slot = max(1 << 16, 2 * _tree_nbytes(probe) + (1 << 16))
        name = f"/pha_dl_{os.getpid()}_{id(self) & 0xffffff}_{np.random.randint(1 << 30)}"
        try:
            return native.ShmRing(name, self.num_workers * self.prefetch_factor, slot)
        except OSError:
            return None

    def __iter__(self):
        dev = self.device
        host = self._host_batches()
        if not self.use_buffer_reader or dev.type != "cuda":
            for b in host:
                yield _to_device_tree(b, dev, False)
            return
        # one-batch-ahead H2D prefetch on a side stream
        stream = torch.cuda.Stream(dev)
        nxt = None
        for b in host:
            with torch.cuda.stream(stream):
                cur = _to_device_tree(b, dev, True)
            _record_stream_tree(cur, torch.cuda.current_stream(dev))
            if nxt is not None:
                yield nxt
            torch.cuda.current_stream(dev).wait_stream(stream)
            nxt = cur
        if nxt is not None:
            yield nxt

    @staticmethod
    def from_generator(feed_list=None, capacity=None, use_double_buffer=True, iterable=True, return_list=False,
                       use_multiprocess=False, drop_last=True):
        return _GeneratorLoader(return_list)


class _GeneratorLoader:
    def __init__(self, return_list):
        self._gen = None
        self.return_list = return_list

    def set_sample_generator(self, reader, batch_size, drop_last=True, places=None):
        def gen():
            batch = []
            for s in reader():
                batch.append(s)
                if len(batch) == batch_size:
                    yield default_collate_fn(batch)
                    batch = []
            if batch and not drop_last:
                yield default_collate_fn(batch)
        self._gen = gen

    def set_sample_list_generator(self, reader, places=None):
        self._gen = lambda: (default_collate_fn(b) for b in reader())

    def set_batch_generator(self, reader, places=None):
        self._gen = reader

    def __iter__(self):
        dev = default_device()
        for b in self._gen():
            yield _to_device_tree(b, dev, False)
