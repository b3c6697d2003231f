"""Legacy reader decorators (reference: python/paddle/reader/decorator.py, paddle.batch)."""
from __future__ import annotations

import itertools
import queue
import random
import threading

__all__ = ["batch", "shuffle", "buffered", "compose", "chain", "firstn", "xmap_readers", "map_readers", "cache",
           "multiprocess_reader", "ComposeNotAligned"]


def batch(reader, batch_size, drop_last=False):
    if batch_size <= 0:
        raise ValueError(f"batch_size should be a positive integer value, but got batch_size={batch_size}")

    def batch_reader():
        b = []
        for inst in reader():
            b.append(inst)
            if len(b) == batch_size:
                yield b
                b = []
        if b and not drop_last:
            yield b
    return batch_reader


def cache(reader):
    all_data = tuple(reader())

    def r():
        yield from all_data
    return r


def map_readers(func, *readers):
    def r():
        for e in zip(*[rd() for rd in readers]):
            yield func(*e)
    return r


def shuffle(reader, buf_size):
    def r():
        buf = []
        for e in reader():
            buf.append(e)
            if len(buf) >= buf_size:
                random.shuffle(buf)
                yield from buf
                buf = []
        random.shuffle(buf)
        yield from buf
    return r


def chain(*readers):
    def r():
        for rd in readers:
            yield from rd()
    return r


class ComposeNotAligned(ValueError):
    pass


def compose(*readers, **kwargs):
    check_alignment = kwargs.pop("check_alignment", True)

    def make_tuple(x):
        return x if isinstance(x, tuple) else (x,)

    def r():
        its = [rd() for rd in readers]
        if not check_alignment:
            for outs in zip(*its):
                yield sum(map(make_tuple, outs), ())
            return
        for outs in itertools.zip_longest(*its):
            if any(o is None for o in outs):
                raise ComposeNotAligned("outputs of readers are not aligned.")
            yield sum(map(make_tuple, outs), ())
    return r


def buffered(reader, size):
    end = object()

    def r():
        q = queue.Queue(maxsize=size)

        def fill():
            for d in reader():
                q.put(d)
            q.put(end)
        threading.Thread(target=fill, daemon=True).start()
        while True:
            e = q.get()
            if e is end:
                return
            yield e
    return r


def firstn(reader, n):
    def r():
        for i, item in enumerate(reader()):
            if i == n:
                break
            yield item
    return r


def xmap_readers(mapper, reader, process_num, buffer_size, order=False):
    """Map with ``process_num`` threads; ``order`` keeps input order."""
    import concurrent.futures as cf

    def r():
        with cf.ThreadPoolExecutor(process_num) as ex:
            if order:
                yield from ex.map(mapper, reader())
            else:
                futs = set()
                for s in reader():
                    futs.add(ex.submit(mapper, s))
                    if len(futs) >= buffer_size:
                        done, futs = cf.wait(futs, return_when=cf.FIRST_COMPLETED)
                        for f in done:
                            yield f.result()
                for f in cf.as_completed(futs):
                    yield f.result()
    return r


def multiprocess_reader(readers, use_pipe=True, queue_size=1000):
    import multiprocessing as mp
    end = "__pha_end__"

    def work(rd, q):
        for s in rd():
            q.put(s)
        q.put(end)

    def r():
        q = mp.get_context("fork").Queue(queue_size)
        ps = [mp.get_context("fork").Process(target=work, args=(rd, q), daemon=True) for rd in readers]
        for p in ps:
            p.start()
        done = 0
        while done < len(readers):
            s = q.get()
            if isinstance(s, str) and s == end:
                done += 1
                continue
            yield s
        for p in ps:
            p.join()
    return r
