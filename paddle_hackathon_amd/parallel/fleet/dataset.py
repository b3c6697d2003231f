"""File-based datasets for ``Executor.train_from_dataset`` / fleet (reference:
python/paddle/distributed/fleet/dataset/dataset.py with the C++ MultiSlot data feed in
paddle/fluid/framework/data_feed.cc and data_set.cc).

Files are read (optionally through ``pipe_command``, a UNIX filter run per file exactly like
the reference), parsed by the native MultiSlot parser (csrc/runtime/datafeed.cpp) and
batched into padded tensors per slot, plus ``<slot>.lod`` offsets when a slot is
variable-length. ``InMemoryDataset`` keeps all instances resident (288 GB HBM-class hosts
make this the common case) and supports local/global shuffle; ``QueueDataset`` streams
file by file."""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess

import numpy as np
import torch

from ...framework.core import Tensor, _wrap, default_device

__all__ = ["DatasetBase", "InMemoryDataset", "QueueDataset", "FileInstantDataset"]


def _var_info(v):
    name = getattr(v, "name", None) or str(v)
    dt = getattr(v, "dtype", "float32")
    dts = str(dt).lower()
    is_float = "float" in dts
    return name, is_float


class DatasetBase:
    def __init__(self):
        self.batch_size = 1
        self.thread_num = 1
        self.use_var = []
        self.pipe_command = "cat"
        self.input_type = 0
        self.filelist = []
        self.drop_last = False

    def init(self, batch_size=1, thread_num=1, use_var=None, pipe_command="cat", input_type=0, fs_name="", fs_ugi="",
             download_cmd="cat", **kwargs):
        self.batch_size = batch_size
        self.thread_num = max(1, thread_num)
        self.use_var = list(use_var or [])
        self.pipe_command = pipe_command
        self.input_type = input_type
        self.download_cmd = download_cmd

    def set_filelist(self, filelist):
        self.filelist = list(filelist)

    def set_batch_size(self, batch_size):
        self.batch_size = batch_size

    def set_thread(self, thread_num):
        self.thread_num = thread_num

    def set_use_var(self, var_list):
        self.use_var = list(var_list)

    def set_pipe_command(self, pipe_command):
        self.pipe_command = pipe_command

    def _slots(self):
        return [_var_info(v) for v in self.use_var]

    def _read_file(self, path):
        if self.pipe_command in (None, "", "cat"):
            with open(path, "rb") as f:
                return f.read()
        with open(path, "rb") as f:
            r = subprocess.run(self.pipe_command, shell=True, stdin=f, stdout=subprocess.PIPE, check=True)
        return r.stdout

    def _parse(self, data):
        from ...utils import native
        slots = self._slots()
        ninst, nbad, cols = native.parse_multislot(data, [f for _, f in slots], self.thread_num)
        return ninst, cols

    def _batches_from(self, ninst, cols, order=None):
        slots = self._slots()
        order = np.arange(ninst) if order is None else order
        dev = default_device()
        bs = self.batch_size
        for start in range(0, ninst, bs):
            idx = order[start:start + bs]
            if len(idx) < bs and self.drop_last:
                break
            batch = {}
            for (name, is_float), (vals, lod) in zip(slots, cols):
                lens = lod[idx + 1] - lod[idx]
                width = int(lens.max()) if len(lens) else 0
                dense = np.zeros((len(idx), max(width, 1)), dtype=vals.dtype)
                for r, i in enumerate(idx):
                    seg = vals[lod[i]:lod[i + 1]]
                    dense[r, :len(seg)] = seg
                batch[name] = _wrap(torch.from_numpy(dense).to(dev))
                if len(lens) and not (lens == lens[0]).all():
                    batch[name + ".lod"] = _wrap(torch.from_numpy(np.concatenate([[0], np.cumsum(lens)])).to(dev))
            yield batch

    def _desc(self):
        return f"{type(self).__name__}(files={len(self.filelist)}, slots={[n for n, _ in self._slots()]})"


class InMemoryDataset(DatasetBase):
    def __init__(self):
        super().__init__()
        self._ninst = 0
        self._cols = None
        self._order = None
        self._shuffled = 0
        self.parse_ins_id = False
        self.parse_content = False
        self.merge_by_lineid = False
        self.fleet_send_batch_size = None

    def _init_distributed_settings(self, **kwargs):
        for k, v in kwargs.items():
            setattr(self, k, v)

    def update_settings(self, **kwargs):
        for k, v in kwargs.items():
            setattr(self, k, v)

    def init(self, **kwargs):
        dist_keys = ("merge_size", "parse_ins_id", "parse_content", "fleet_send_batch_size", "fleet_send_sleep_seconds",
                     "fea_eval", "candidate_size")
        self._init_distributed_settings(**{k: kwargs.pop(k) for k in list(kwargs) if k in dist_keys})
        super().init(**kwargs)

    def load_into_memory(self, is_shuffle=False):
        with cf.ThreadPoolExecutor(max_workers=self.thread_num) as ex:
            blobs = list(ex.map(self._read_file, self.filelist))
        ninst, cols = self._parse(b"".join(b if b.endswith(b"\n") or not b else b + b"\n" for b in blobs))
        self._ninst, self._cols = ninst, cols
        self._order = np.arange(ninst)
        if is_shuffle:
            self.local_shuffle()

    def preload_into_memory(self, thread_num=None):
        import threading
        if thread_num:
            self.thread_num = thread_num
        self._preload = threading.Thread(target=self.load_into_memory)
        self._preload.start()

    def wait_preload_done(self):
        t = getattr(self, "_preload", None)
        if t is not None:
            t.join()
            self._preload = None

    def local_shuffle(self):
        self._order = np.random.permutation(self._ninst)

    def global_shuffle(self, fleet=None, thread_num=12):
        """Redistribute instances uniformly at random across trainers (all-to-all of instances)."""
        import torch.distributed as dist
        if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
            self.local_shuffle()
            return
        world, me = dist.get_world_size(), dist.get_rank()
        dest = np.random.randint(0, world, size=self._ninst)
        outgoing = []
        for r in range(world):
            idx = np.nonzero(dest == r)[0]
            outgoing.append([[vals[lod[i]:lod[i + 1]] for i in idx] for vals, lod in self._cols])
        gathered = [None] * world
        dist.all_gather_object(gathered, outgoing)
        mine = [g[me] for g in gathered]
        cols = []
        for s in range(len(self._cols)):
            segs = [seg for part in mine for seg in part[s]]
            lod = np.concatenate([[0], np.cumsum([len(x) for x in segs])]).astype(np.int64)
            vals = np.concatenate(segs) if segs else self._cols[s][0][:0]
            cols.append((vals, lod))
        self._cols = cols
        self._ninst = len(cols[0][1]) - 1 if cols else 0
        self._order = np.random.permutation(self._ninst)
        self._shuffled = self._ninst

    def release_memory(self):
        self._cols, self._ninst, self._order = None, 0, None

    def get_memory_data_size(self, fleet=None):
        import torch.distributed as dist
        n = torch.tensor([self._ninst])
        if dist.is_available() and dist.is_initialized():
            dist.all_reduce(n)
        return int(n.item())

    def get_shuffle_data_size(self, fleet=None):
        import torch.distributed as dist
        n = torch.tensor([self._shuffled])
        if dist.is_available() and dist.is_initialized():
            dist.all_reduce(n)
        return int(n.item())

    def slots_shuffle(self, slots):
        """Shuffle the values of the named slots across instances (feature importance eval)."""
        names = [n for n, _ in self._slots()]
        for s in slots:
            k = names.index(s)
            vals, lod = self._cols[k]
            perm = np.random.permutation(self._ninst)
            segs = [vals[lod[i]:lod[i + 1]] for i in perm]
            lod2 = np.concatenate([[0], np.cumsum([len(x) for x in segs])]).astype(np.int64)
            self._cols[k] = (np.concatenate(segs) if segs else vals[:0], lod2)

    def __iter__(self):
        if self._cols is None:
            raise RuntimeError("call load_into_memory() first")
        yield from self._batches_from(self._ninst, self._cols, self._order)

    def __len__(self):
        return (self._ninst + self.batch_size - 1) // self.batch_size


class QueueDataset(DatasetBase):
    """Streams files one at a time (no global shuffle), reading the next file in background."""

    def init(self, **kwargs):
        super().init(**kwargs)

    def __iter__(self):
        with cf.ThreadPoolExecutor(max_workers=1) as ex:
            fut = ex.submit(self._read_file, self.filelist[0]) if self.filelist else None
            for k in range(len(self.filelist)):
                data = fut.result()
                fut = ex.submit(self._read_file, self.filelist[k + 1]) if k + 1 < len(self.filelist) else None
                ninst, cols = self._parse(data)
                yield from self._batches_from(ninst, cols)

    def local_shuffle(self):
        raise NotImplementedError("QueueDataset does not support local shuffle")

    def global_shuffle(self, fleet=None):
        raise NotImplementedError("QueueDataset does not support global shuffle")


class FileInstantDataset(QueueDataset):
    pass
