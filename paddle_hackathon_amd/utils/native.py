"""ctypes bindings for the host C++ runtime ``_C/libpha_runtime.so`` (csrc/runtime/*.cpp).

Everything here has a pure-Python fallback so CPU-only environments without a compiler still
work; ``available()`` says whether the native path is in use.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_LIB_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_C", "libpha_runtime.so")
_lib = None
_tried = False

_c_i64p = ctypes.POINTER(ctypes.c_int64)
_c_i32p = ctypes.POINTER(ctypes.c_int32)
_c_u8p = ctypes.POINTER(ctypes.c_uint8)


def _load():
    global _lib, _tried
    if _tried:
        return _lib
    _tried = True
    if not os.path.exists(_LIB_PATH):
        return None
    try:
        lib = ctypes.CDLL(_LIB_PATH)
    except OSError:
        return None
    sig = {
        "pha_stack_arrays": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int64, ctypes.c_size_t,
                                            ctypes.c_void_p, ctypes.c_int]),
        "pha_gather_rows": (ctypes.c_int, [ctypes.c_void_p, _c_i64p, ctypes.c_int64, ctypes.c_size_t, ctypes.c_void_p,
                                           ctypes.c_int]),
        "pha_runtime_version": (ctypes.c_int, []),
        "pha_plan_buckets": (ctypes.c_int, [ctypes.c_int64, _c_i64p, _c_i32p, _c_u8p, _c_i64p, ctypes.c_int, _c_i64p,
                                            _c_i32p]),
        "pha_bucket_padded_numel": (ctypes.c_int64, [ctypes.c_int64, ctypes.c_int64, ctypes.c_int64]),
        "pha_tracer_enable": (None, [ctypes.c_int]),
        "pha_tracer_enabled": (ctypes.c_int, []),
        "pha_tracer_now_ns": (ctypes.c_int64, []),
        "pha_tracer_push": (None, [ctypes.c_char_p, ctypes.c_int32]),
        "pha_tracer_pop": (None, []),
        "pha_tracer_record": (None, [ctypes.c_char_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_int64]),
        "pha_tracer_count": (ctypes.c_int64, []),
        "pha_tracer_clear": (None, []),
        "pha_tracer_export_chrome": (ctypes.c_int64, [ctypes.c_char_p, ctypes.c_int64]),
        "pha_arena_create": (ctypes.c_void_p, [ctypes.c_int64, ctypes.c_int64]),
        "pha_arena_destroy": (None, [ctypes.c_void_p]),
        "pha_arena_alloc": (ctypes.c_int64, [ctypes.c_void_p, ctypes.c_int64]),
        "pha_arena_free": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64]),
        "pha_arena_used": (ctypes.c_int64, [ctypes.c_void_p]),
        "pha_arena_peak": (ctypes.c_int64, [ctypes.c_void_p]),
        "pha_arena_capacity": (ctypes.c_int64, [ctypes.c_void_p]),
        "pha_arena_largest_free": (ctypes.c_int64, [ctypes.c_void_p]),
        "pha_arena_num_free_blocks": (ctypes.c_int64, [ctypes.c_void_p]),
        "pha_plan_memory": (ctypes.c_int64, [ctypes.c_int64, _c_i64p, _c_i64p, _c_i64p, ctypes.c_int64, _c_i64p]),
        "pha_ring_create": (ctypes.c_void_p, [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint64]),
        "pha_ring_attach": (ctypes.c_void_p, [ctypes.c_char_p]),
        "pha_ring_nslots": (ctypes.c_uint32, [ctypes.c_void_p]),
        "pha_ring_slot_bytes": (ctypes.c_uint64, [ctypes.c_void_p]),
        "pha_ring_slot_ptr": (ctypes.c_void_p, [ctypes.c_void_p, ctypes.c_uint32]),
        "pha_ring_slot_nbytes": (ctypes.c_uint64, [ctypes.c_void_p, ctypes.c_uint32]),
        "pha_ring_acquire_write": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
        "pha_ring_commit": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int64, ctypes.c_uint64]),
        "pha_ring_abort": (None, [ctypes.c_void_p, ctypes.c_uint32]),
        "pha_ring_acquire_read": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int]),
        "pha_ring_release": (None, [ctypes.c_void_p, ctypes.c_uint32]),
        "pha_ring_ready_count": (ctypes.c_int, [ctypes.c_void_p]),
        "pha_ring_close": (None, [ctypes.c_void_p]),
        "pha_ring_destroy": (None, [ctypes.c_void_p]),
        "pha_ring_detach": (None, [ctypes.c_void_p]),
        "pha_ms_parse": (ctypes.c_void_p, [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, _c_u8p, ctypes.c_int]),
        "pha_ms_ninst": (ctypes.c_int64, [ctypes.c_void_p]),
        "pha_ms_nbad": (ctypes.c_int64, [ctypes.c_void_p]),
        "pha_ms_slot_numel": (ctypes.c_int64, [ctypes.c_void_p, ctypes.c_int]),
        "pha_ms_copy": (None, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, _c_i64p]),
        "pha_ms_free": (None, [ctypes.c_void_p]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _lib = lib
    return lib


def available():
    return _load() is not None


def lib():
    l = _load()
    if l is None:
        raise RuntimeError(f"native runtime {_LIB_PATH} not built (python -m paddle_hackathon_amd.ops.build)")
    return l


def _ptr(a, t):
    return a.ctypes.data_as(t)


# ----------------------------------------------------------------------------- collate
def stack_arrays(arrs, out=None):
    """np.stack for equally-shaped contiguous arrays, copied by the native thread pool."""
    a0 = np.ascontiguousarray(arrs[0])
    l = _load()
    if l is None:
        return np.stack(arrs, out=out)
    arrs = [a if (a.flags.c_contiguous and a.dtype == a0.dtype and a.shape == a0.shape) else None
            for a in (np.asarray(x) for x in arrs)]
    if any(a is None for a in arrs):
        return np.stack(arrs, out=out)
    if out is None:
        out = np.empty((len(arrs),) + a0.shape, dtype=a0.dtype)
    ptrs = (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
    rc = l.pha_stack_arrays(ptrs, len(arrs), a0.nbytes, out.ctypes.data, 0)
    if rc != 0:
        raise RuntimeError("pha_stack_arrays failed")
    return out


def gather_rows(src, idx, out=None):
    src = np.ascontiguousarray(src)
    idx = np.ascontiguousarray(idx, dtype=np.int64)
    if idx.size and (idx.min() < 0 or idx.max() >= src.shape[0]):
        raise IndexError("gather_rows index out of range")
    l = _load()
    if l is None:
        return np.take(src, idx, axis=0, out=out)
    if out is None:
        out = np.empty((idx.size,) + src.shape[1:], dtype=src.dtype)
    row = src[0].nbytes if src.shape[0] else 0
    l.pha_gather_rows(src.ctypes.data, _ptr(idx, _c_i64p), idx.size, row, out.ctypes.data, 0)
    return out


# ----------------------------------------------------------------------------- buckets
def plan_buckets(nbytes, dtype_ids, limits, is_sparse=None, order=None):
    """Assign each tensor a bucket id (see csrc/runtime/bucket.cpp). Returns list[int]."""
    n = len(nbytes)
    if n == 0:
        return []
    nb = np.asarray(nbytes, dtype=np.int64)
    dt = np.asarray(dtype_ids, dtype=np.int32)
    lim = np.asarray(limits, dtype=np.int64)
    sp = np.asarray(is_sparse if is_sparse is not None else [0] * n, dtype=np.uint8)
    od = np.asarray(order if order is not None else range(n), dtype=np.int64)
    out = np.full(n, -1, dtype=np.int32)
    l = _load()
    if l is not None:
        ng = l.pha_plan_buckets(n, _ptr(nb, _c_i64p), _ptr(dt, _c_i32p), _ptr(sp, _c_u8p), _ptr(lim, _c_i64p), len(lim),
                                _ptr(od, _c_i64p), _ptr(out, _c_i32p))
        if ng < 0:
            raise ValueError("invalid bucket plan arguments")
        return out.tolist()
    # python fallback, same algorithm
    open_, gid, cursor = {}, 0, 0
    for i in od:
        if sp[i]:
            out[i] = gid
            gid += 1
            continue
        b = open_.get(int(dt[i]))
        if b is not None:
            limv = lim[min(b[2], len(lim) - 1)]
            if b[1] + nb[i] <= limv or b[1] == 0:
                b[1] += nb[i]
                out[i] = b[0]
                continue
        open_[int(dt[i])] = [gid, int(nb[i]), cursor]
        out[i] = gid
        gid += 1
        cursor += 1
    return out.tolist()


def bucket_padded_numel(numel, world, align_elems=8):
    unit = max(1, world) * max(1, align_elems)
    return (numel + unit - 1) // unit * unit


# ----------------------------------------------------------------------------- tracer
class HostTracer:
    """Thin wrapper over the native host tracer (falls back to a Python list)."""
    TYPES = {"UserDefined": 0, "Operator": 1, "Dataloader": 2, "ProfileStep": 3, "Forward": 4, "Backward": 5,
             "Optimization": 6, "Communication": 7, "PythonOp": 8}

    def __init__(self):
        self._l = _load()
        self._py_events = []
        self._py_stack = []
        self._enabled = False

    def enable(self, on=True):
        self._enabled = bool(on)
        if self._l is not None:
            self._l.pha_tracer_enable(1 if on else 0)

    @property
    def enabled(self):
        return self._enabled

    def push(self, name, type_name="UserDefined"):
        if not self._enabled:
            return
        t = self.TYPES.get(type_name, 0)
        if self._l is not None:
            self._l.pha_tracer_push(name.encode(), t)
        else:
            import time
            self._py_stack.append((name, t, time.time_ns()))

    def pop(self):
        if self._l is not None:
            self._l.pha_tracer_pop()
        elif self._py_stack:
            import time
            name, t, s = self._py_stack.pop()
            if self._enabled:
                self._py_events.append((name, t, s, time.time_ns()))

    def record(self, name, type_name, start_ns, end_ns):
        if not self._enabled:
            return
        t = self.TYPES.get(type_name, 0)
        if self._l is not None:
            self._l.pha_tracer_record(name.encode(), t, int(start_ns), int(end_ns))
        else:
            self._py_events.append((name, t, int(start_ns), int(end_ns)))

    def count(self):
        return self._l.pha_tracer_count() if self._l is not None else len(self._py_events)

    def clear(self):
        if self._l is not None:
            self._l.pha_tracer_clear()
        self._py_events.clear()

    def export_chrome(self, path, pid=None):
        pid = os.getpid() if pid is None else pid
        if self._l is not None:
            n = self._l.pha_tracer_export_chrome(path.encode(), pid)
            if n < 0:
                raise OSError(f"cannot write {path}")
            return n
        import json
        inv = {v: k for k, v in self.TYPES.items()}
        ev = [{"name": n, "cat": inv.get(t, "UserDefined"), "ph": "X", "pid": pid, "tid": 0, "ts": s / 1e3,
               "dur": (e - s) / 1e3} for n, t, s, e in self._py_events]
        with open(path, "w") as f:
            json.dump({"traceEvents": ev, "displayTimeUnit": "ms"}, f)
        return len(ev)


_tracer = None


def host_tracer():
    global _tracer
    if _tracer is None:
        _tracer = HostTracer()
    return _tracer


# ----------------------------------------------------------------------------- arena / planner
class Arena:
    """Best-fit coalescing offset allocator over [0, capacity) (csrc/runtime/arena.cpp)."""

    def __init__(self, capacity, alignment=256):
        self._h = lib().pha_arena_create(int(capacity), int(alignment))
        if not self._h:
            raise ValueError("invalid arena capacity")

    def alloc(self, nbytes):
        off = lib().pha_arena_alloc(self._h, int(nbytes))
        if off < 0:
            raise MemoryError(f"arena out of memory for {nbytes} bytes (largest free {self.largest_free})")
        return off

    def free(self, off):
        if lib().pha_arena_free(self._h, int(off)) != 0:
            raise ValueError(f"offset {off} is not a live allocation")

    used = property(lambda s: lib().pha_arena_used(s._h))
    peak = property(lambda s: lib().pha_arena_peak(s._h))
    capacity = property(lambda s: lib().pha_arena_capacity(s._h))
    largest_free = property(lambda s: lib().pha_arena_largest_free(s._h))
    num_free_blocks = property(lambda s: lib().pha_arena_num_free_blocks(s._h))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _lib is not None:
            _lib.pha_arena_destroy(h)
            self._h = None


def plan_memory(sizes, first_use, last_use, alignment=256):
    """Lifetime-based static memory plan; returns (offsets list, total bytes)."""
    n = len(sizes)
    s = np.asarray(sizes, dtype=np.int64)
    f = np.asarray(first_use, dtype=np.int64)
    e = np.asarray(last_use, dtype=np.int64)
    out = np.zeros(n, dtype=np.int64)
    total = lib().pha_plan_memory(n, _ptr(s, _c_i64p), _ptr(f, _c_i64p), _ptr(e, _c_i64p), alignment,
                                  _ptr(out, _c_i64p))
    return out.tolist(), int(total)


# ----------------------------------------------------------------------------- shm ring
class ShmRing:
    """Shared-memory slot ring (csrc/runtime/shm_ring.cpp) for DataLoader worker → trainer batches."""

    def __init__(self, name, nslots=None, slot_bytes=None, create=True):
        self.name = name if name.startswith("/") else "/" + name
        l = lib()
        self._h = l.pha_ring_create(self.name.encode(), nslots, slot_bytes) if create else \
            l.pha_ring_attach(self.name.encode())
        if not self._h:
            raise OSError(f"cannot {'create' if create else 'attach'} shared-memory ring {self.name}")
        self.owner = create
        self.nslots = l.pha_ring_nslots(self._h)
        self.slot_bytes = l.pha_ring_slot_bytes(self._h)

    def slot_view(self, i, nbytes=None):
        p = lib().pha_ring_slot_ptr(self._h, i)
        n = self.slot_bytes if nbytes is None else nbytes
        return np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(p))

    def acquire_write(self, timeout_ms=-1):
        return lib().pha_ring_acquire_write(self._h, int(timeout_ms))

    def commit(self, i, seq, nbytes):
        if lib().pha_ring_commit(self._h, i, int(seq), int(nbytes)) != 0:
            raise ValueError(f"payload of {nbytes} bytes exceeds slot size {self.slot_bytes}")

    def abort(self, i):
        lib().pha_ring_abort(self._h, i)

    def acquire_read(self, seq, timeout_ms=-1):
        return lib().pha_ring_acquire_read(self._h, int(seq), int(timeout_ms))

    def nbytes(self, i):
        return lib().pha_ring_slot_nbytes(self._h, i)

    def release(self, i):
        lib().pha_ring_release(self._h, i)

    def ready_count(self):
        return lib().pha_ring_ready_count(self._h)

    def close(self):
        if self._h:
            lib().pha_ring_close(self._h)

    def destroy(self):
        if self._h:
            (lib().pha_ring_destroy if self.owner else lib().pha_ring_detach)(self._h)
            self._h = None

    def detach(self):
        """Unmap without unlinking (forked children holding the creator's handle)."""
        if self._h:
            lib().pha_ring_detach(self._h)
            self._h = None


# --------------------------------------------------------------------------- payload codec
_ALIGN = 64


def pack_into(tree, buf):
    """Serialise a tree of numpy arrays/scalars into ``buf`` (uint8 array).
    Layout: [u64 meta_len][pickle meta][pad to 64][array bytes, each 64-aligned]; array
    offsets in the meta are relative to the data region. Returns bytes used, or -needed
    if ``buf`` is too small (nothing is written then)."""
    import pickle
    arrays = []

    def strip(x):
        if isinstance(x, np.ndarray):
            arrays.append(np.ascontiguousarray(x))
            return ("__pha_arr__", len(arrays) - 1, x.dtype.str, x.shape)
        if isinstance(x, dict):
            return {k: strip(v) for k, v in x.items()}
        if isinstance(x, (list, tuple)):
            return type(x)(strip(v) for v in x)
        return x

    tree = strip(tree)
    rel, off = [], 0
    for a in arrays:
        rel.append(off)
        off = (off + a.nbytes + _ALIGN - 1) // _ALIGN * _ALIGN
    meta = pickle.dumps((rel, tree), protocol=4)
    head = (8 + len(meta) + _ALIGN - 1) // _ALIGN * _ALIGN
    end = head + (rel[-1] + arrays[-1].nbytes if arrays else 0)
    if end > buf.size:
        return -end
    buf[:8] = np.frombuffer(np.uint64(len(meta)).tobytes(), np.uint8)
    buf[8:8 + len(meta)] = np.frombuffer(meta, np.uint8)
    for a, o in zip(arrays, rel):
        buf[head + o:head + o + a.nbytes] = a.reshape(-1).view(np.uint8)
    return end


def unpack_from(buf, copy=True):
    """Inverse of :func:`pack_into`. With ``copy=False`` arrays are views into ``buf``."""
    import pickle
    n = int(np.frombuffer(buf[:8].tobytes(), np.uint64)[0])
    rel, tree = pickle.loads(buf[8:8 + n].tobytes())
    head = (8 + n + _ALIGN - 1) // _ALIGN * _ALIGN

    def build(x):
        if isinstance(x, tuple) and len(x) == 4 and x[0] == "__pha_arr__":
            _, i, dt, shape = x
            dt = np.dtype(dt)
            nb = int(np.prod(shape, dtype=np.int64)) * dt.itemsize
            a = buf[head + rel[i]:head + rel[i] + nb].view(dt).reshape(shape)
            return a.copy() if copy else a
        if isinstance(x, dict):
            return {k: build(v) for k, v in x.items()}
        if isinstance(x, (list, tuple)):
            return type(x)(build(v) for v in x)
        return x

    return build(tree)


# ----------------------------------------------------------------------------- MultiSlot parser
def parse_multislot(data: bytes, slot_is_float, nthreads=0):
    """Parse MultiSlot text (``<n> v1..vn`` per slot per line). Returns
    (ninst, nbad, [(values ndarray, lod ndarray), ...]) — values float32 or int64 per slot."""
    n = len(slot_is_float)
    isf = np.asarray([1 if f else 0 for f in slot_is_float], dtype=np.uint8)
    l = _load()
    if l is None:
        return _parse_multislot_py(data, isf)
    h = l.pha_ms_parse(data, len(data), n, _ptr(isf, _c_u8p), int(nthreads))
    try:
        ninst, nbad = l.pha_ms_ninst(h), l.pha_ms_nbad(h)
        out = []
        for s in range(n):
            vals = np.empty(l.pha_ms_slot_numel(h, s), dtype=np.float32 if isf[s] else np.int64)
            lod = np.empty(ninst + 1, dtype=np.int64)
            l.pha_ms_copy(h, s, vals.ctypes.data, _ptr(lod, _c_i64p))
            out.append((vals, lod))
        return ninst, nbad, out
    finally:
        l.pha_ms_free(h)


def _parse_multislot_py(data, isf):
    n = len(isf)
    vals = [[] for _ in range(n)]
    lods = [[0] for _ in range(n)]
    ninst = nbad = 0
    for line in data.decode().splitlines():
        tok = line.split()
        if not tok:
            continue
        pos, rec = 0, []
        try:
            for s in range(n):
                k = int(tok[pos])
                pos += 1
                conv = float if isf[s] else int
                rec.append([conv(t) for t in tok[pos:pos + k]])
                if len(rec[-1]) != k:
                    raise ValueError
                pos += k
        except (ValueError, IndexError):
            nbad += 1
            continue
        for s in range(n):
            vals[s].extend(rec[s])
            lods[s].append(len(vals[s]))
        ninst += 1
    return ninst, nbad, [(np.asarray(v, dtype=np.float32 if isf[s] else np.int64), np.asarray(lods[s], dtype=np.int64))
                         for s, v in enumerate(vals)]
