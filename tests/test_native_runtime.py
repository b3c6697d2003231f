"""Native C++ runtime (csrc/runtime): collate, gather, bucket planner, arena + memory
planner, host tracer, shared-memory ring, MultiSlot parser — each vs a Python reference."""
import multiprocessing as mp
import os

import numpy as np
import pytest

from paddle_hackathon_amd.utils import native as N


@pytest.fixture(scope="module", autouse=True)
def _built():
    from paddle_hackathon_amd.ops.build import build_runtime
    build_runtime(verbose=False)
    N._tried, N._lib = False, None
    assert N.available()


def test_stack_and_gather():
    small = [np.random.rand(3, 4).astype("f4") for _ in range(5)]
    np.testing.assert_array_equal(N.stack_arrays(small), np.stack(small))
    big = [np.random.rand(128, 1024).astype("f4") for _ in range(16)]  # > 1 MiB: threaded path
    np.testing.assert_array_equal(N.stack_arrays(big), np.stack(big))
    src = np.random.rand(100, 7)
    idx = np.random.randint(0, 100, 50)
    np.testing.assert_array_equal(N.gather_rows(src, idx), src[idx])
    with pytest.raises(IndexError):
        N.gather_rows(src, [100])


def test_bucket_planner_matches_python():
    rng = np.random.RandomState(0)
    for _ in range(20):
        n = rng.randint(1, 40)
        nb = rng.randint(1, 100, n).tolist()
        dt = rng.randint(0, 3, n).tolist()
        sp = rng.randint(0, 2, n).tolist()
        lim = [rng.randint(50, 200), rng.randint(100, 400)]
        order = rng.permutation(n).tolist()
        native = N.plan_buckets(nb, dt, lim, sp, order)
        lib, N._lib = N._lib, None
        N._tried = True
        try:
            py = N.plan_buckets(nb, dt, lim, sp, order)
        finally:
            N._lib = lib
        assert native == py
        # a bucket never mixes dtypes, sparse tensors are alone
        for g in set(native):
            members = [i for i in range(n) if native[i] == g]
            assert len({dt[i] for i in members}) == 1
            if any(sp[i] for i in members):
                assert len(members) == 1
    assert N.bucket_padded_numel(10, 4, 8) == 32


def test_arena_best_fit_and_coalesce():
    a = N.Arena(1 << 20, 256)
    offs = [a.alloc(1000) for _ in range(4)]
    assert offs == [0, 1024, 2048, 3072]
    a.free(offs[1])
    a.free(offs[2])  # coalesces with the previous hole
    assert a.alloc(2000) == 1024  # best fit lands in the merged 2048-byte hole
    a.free(offs[0])
    a.free(offs[3])
    assert a.peak == 4096
    with pytest.raises(MemoryError):
        a.alloc(2 << 20)
    with pytest.raises(ValueError):
        a.free(12345)


def test_memory_plan_no_overlap():
    rng = np.random.RandomState(1)
    n = 30
    sizes = rng.randint(1, 5000, n)
    first = rng.randint(0, 20, n)
    last = first + rng.randint(0, 10, n)
    offs, total = N.plan_memory(sizes, first, last, 256)
    r = lambda s: (s + 255) // 256 * 256  # noqa: E731
    for i in range(n):
        for j in range(i + 1, n):
            if not (last[i] < first[j] or last[j] < first[i]):
                assert offs[i] + r(sizes[i]) <= offs[j] or offs[j] + r(sizes[j]) <= offs[i]
    assert total <= sum(r(s) for s in sizes)
    peak_live = max(sum(r(sizes[i]) for i in range(n) if first[i] <= t <= last[i]) for t in range(30))
    assert total >= peak_live


def test_tracer_chrome_export(tmp_path):
    tr = N.HostTracer()
    tr.clear()
    tr.enable(True)
    tr.push("outer", "Forward")
    tr.push("inner \"q\"", "Operator")
    tr.pop()
    tr.pop()
    tr.record("manual", "Communication", 1000, 5000)
    tr.enable(False)
    tr.push("ignored")
    tr.pop()
    p = str(tmp_path / "t.json")
    assert tr.export_chrome(p) == 3
    import json
    ev = json.load(open(p))["traceEvents"]
    names = {e["name"]: e for e in ev}
    assert names["manual"]["dur"] == pytest.approx(4.0)
    assert names["inner \"q\""]["cat"] == "Operator"
    assert names["outer"]["dur"] >= names["inner \"q\""]["dur"]
    tr.clear()


def _producer(name, seqs):
    r = N.ShmRing(name, create=False)
    for s in seqs:
        slot = r.acquire_write(5000)
        assert slot >= 0
        n = N.pack_into({"x": np.full((4, 3), s, np.float32), "s": s}, r.slot_view(slot))
        r.commit(slot, s, n)
    r.detach()


@pytest.mark.parametrize("nslots,nprod", [(12, 2), (3, 1)])
def test_shm_ring_cross_process_ordering(nslots, nprod):
    # (12, 2): two producers finish out of order, consumer still sees 0..11 in order.
    # (3, 1): ring smaller than the stream, the producer blocks on the futex until slots free.
    # (The DataLoader keeps outstanding batches <= nslots, the deadlock-freedom condition.)
    name = f"/pha_test_{os.getpid()}_{nslots}"
    ring = N.ShmRing(name, nslots=nslots, slot_bytes=1 << 14)
    try:
        ctx = mp.get_context("fork")
        ps = [ctx.Process(target=_producer, args=(name, list(range(w, 12, nprod)))) for w in range(nprod)]
        for p in ps:
            p.start()
        for seq in range(12):
            slot = ring.acquire_read(seq, 10000)
            assert slot >= 0
            got = N.unpack_from(ring.slot_view(slot, ring.nbytes(slot)))
            assert got["s"] == seq and (got["x"] == seq).all()
            ring.release(slot)
        for p in ps:
            p.join(10)
            assert p.exitcode == 0
        assert ring.acquire_read(99, 50) == -1  # timeout
        ring.close()
        assert ring.acquire_write(50) == -2
    finally:
        ring.destroy()
    assert not os.path.exists("/dev/shm" + name)


def test_pack_too_small():
    buf = np.zeros(128, np.uint8)
    assert N.pack_into({"a": np.zeros(1000, np.float32)}, buf) < 0


def test_multislot_parser_native_vs_python():
    data = b"2 1 2 1 0.5\n1 7 2 0.1 0.2\nbad line\n\n3 4 5 6 1 9.0\n"
    nat = N.parse_multislot(data, [False, True])
    py = N._parse_multislot_py(data, np.array([0, 1], np.uint8))
    assert nat[0] == py[0] == 3 and nat[1] == py[1] == 1
    for (a, la), (b, lb) in zip(nat[2], py[2]):
        np.testing.assert_allclose(a, b)
        np.testing.assert_array_equal(la, lb)
    big = b"".join(b"2 %d %d 1 %f\n" % (i, i + 1, i * 0.5) for i in range(100000))
    n, bad, cols = N.parse_multislot(big, [False, True])
    assert n == 100000 and bad == 0
    np.testing.assert_array_equal(cols[0][0][::2], np.arange(100000))
    np.testing.assert_allclose(cols[1][0], np.arange(100000) * 0.5, rtol=1e-6)
