"""GPU parameter server (HBM hash tables sharded over ranks; reference heter_ps HeterComm +
hashtable_kernel.cu + optimizer.cuh.h). CPU/gloo: the owner-routing all-to-all protocol over
the host fallback must equal one process holding the whole table; GPU: the HIP hash table
must match the host fallback bit for bit on init and closely on AdaGrad."""
import numpy as np
import pytest
import torch

from dist_helper import run_dist

pytestmark = pytest.mark.timeout(300)

IDS = [np.array([5, 9, 5, 2, 100, 9, 7]), np.array([9, 3, 3, 100, 42])]
GRADS = [np.random.RandomState(1).randn(7, 4).astype("float32"), np.random.RandomState(2).randn(5, 4).astype("float32")]


def _sharded(rank, world):
    from paddle_hackathon_amd.parallel.ps import GpuPsTable
    t = GpuPsTable(4, 64, lr=0.1, initial_range=0.5, seed=3, device="cpu")
    v0 = t.pull(IDS[rank]).numpy()
    t.push(IDS[rank], GRADS[rank])
    v1 = t.pull(np.concatenate(IDS)).numpy()
    return {"v0": v0, "v1": v1, "size": t.size(), "local": t.local_size()}


@pytest.mark.dist
def test_sharded_table_matches_single_table():
    res = run_dist(_sharded, 2)
    from paddle_hackathon_amd.parallel.ps import GpuPsTable
    ref = GpuPsTable(4, 64, lr=0.1, initial_range=0.5, seed=3, device="cpu")
    r0 = [ref.pull(i).numpy() for i in IDS]
    # both ranks' pushes land on the owners before the second pull: apply them as one push
    ref.push(np.concatenate(IDS), np.concatenate(GRADS))
    r1 = ref.pull(np.concatenate(IDS)).numpy()
    for rank, r in enumerate(res):
        np.testing.assert_allclose(r["v0"], r0[rank], rtol=1e-6)
        np.testing.assert_allclose(r["v1"], r1, rtol=1e-5, atol=1e-6)
        assert r["size"] == len(set(np.concatenate(IDS).tolist()))
    assert res[0]["local"] + res[1]["local"] == res[0]["size"]


def test_host_table_rules():
    from paddle_hackathon_amd.parallel.ps import GpuPsTable
    t = GpuPsTable(3, 8, lr=0.2, initial_g2sum=3.0, initial_range=0.1, seed=1, device="cpu")
    w0 = t.pull([1, 2]).numpy()
    assert np.all(np.abs(w0) <= 0.1) and not np.allclose(w0[0], w0[1])
    np.testing.assert_array_equal(t.pull([1, 2]).numpy(), w0)          # stable
    g = np.array([[1.0, 2.0, 3.0], [0.5, 0.5, 0.5]], np.float32)
    t.push([1, 2, 1], np.concatenate([g, g[:1]]))                       # id 1 twice: summed
    want = w0.copy()
    want[0] -= 0.2 * 2 * g[0]
    want[1] -= 0.2 * g[1]
    np.testing.assert_allclose(t.pull([1, 2]).numpy(), want, rtol=1e-6)
    assert np.all(t.pull([77], training=False).numpy() == 0) and t.local_size() == 2
    with pytest.raises(MemoryError):
        t.pull(np.arange(100, 120))


@pytest.mark.gpu
def test_gpu_hash_table_matches_host():
    from paddle_hackathon_amd.parallel.ps import GpuPsTable
    kw = dict(lr=0.1, initial_range=0.5, seed=7)
    gpu = GpuPsTable(16, 50000, device="cuda", **kw)
    cpu = GpuPsTable(16, 50000, device="cpu", **kw)
    rng = np.random.RandomState(0)
    ids = rng.randint(0, 2 ** 40, 20000)
    ids[:500] = ids[500:1000]                          # duplicates
    a = gpu.pull(ids).cpu().numpy()
    b = cpu.pull(ids).numpy()
    np.testing.assert_array_equal(a, b)                # hash-derived init is identical
    g = rng.randn(ids.size, 16).astype("float32")
    gpu.push(ids, g)
    cpu.push(ids, g)
    np.testing.assert_allclose(gpu.pull(ids).cpu().numpy(), cpu.pull(ids).numpy(), rtol=1e-5, atol=1e-6)
    assert gpu.local_size() == cpu.local_size() == len(set(ids.tolist()))
    np.testing.assert_array_equal(gpu.pull([2 ** 41 + 5], training=False).cpu().numpy(), np.zeros((1, 16)))
    sd = gpu.state_dict()
    again = GpuPsTable(16, 50000, device="cuda", **kw)
    again.set_state_dict(sd)
    np.testing.assert_array_equal(again.pull(ids[:100], training=False).cpu().numpy(), gpu.pull(ids[:100]).cpu().numpy())
