"""Own reshard planning (parallel/auto_parallel/reshard.py; reference auto_parallel/reshard.py):
the per-mesh-dim step plan for layout changes, and its execution on 4 gloo ranks (2 x 2 mesh) for
splits, replications, swaps between mesh dims and partial sums, on local blocks and on DTensors."""
import itertools

import numpy as np
import pytest
import torch

from dist_helper import run_dist

pytestmark = pytest.mark.timeout(240)


def test_plan_steps():
    from paddle_hackathon_amd.parallel.auto_parallel.reshard import plan
    k = lambda st: [(s.kind, s.mesh_dim, s.src, s.dst) for s in st]      # noqa: E731
    assert k(plan([0, -1], [-1, 0], 1)) == [("all_to_all", 0, 0, 1)]
    assert k(plan([0, -1], [-1, -1], 1)) == [("all_gather", 0, 0, None)]
    assert k(plan([-1, -1], [-1, 0], 1)) == [("slice", 0, None, 1)]
    assert k(plan([-1, -1], [0, -1], 1, partial=[0])) == [("reduce_scatter", 0, None, 0)]
    assert k(plan([-1, -1], [-1, -1], 1, partial=[0])) == [("all_reduce", 0, None, None)]
    # swapping two mesh dims between two tensor dims: gathers first, then slices (never nested)
    assert k(plan([0, 1], [1, 0], 2)) == [("all_gather", 0, 0, None), ("all_gather", 1, 1, None),
                                          ("slice", 0, None, 1), ("slice", 1, None, 0)]
    assert plan([0, 1], [0, 1], 2) == []


def _block(A, dm, coord, topo):
    t = A
    for i, m in enumerate(dm):
        if m >= 0:
            n = topo[m]
            sz = t.shape[i] // n
            t = t.narrow(i, coord[m] * sz, sz)
    return t


LAYOUTS = [[-1, -1], [0, -1], [1, -1], [-1, 0], [-1, 1], [0, 1], [1, 0]]


def _worker(rank, world):
    from paddle_hackathon_amd.distributed import auto_parallel as ap
    from paddle_hackathon_amd.parallel.auto_parallel.reshard import plan, execute
    mesh = ap.ProcessMesh([[0, 1], [2, 3]], dim_names=["x", "y"])
    coord = [int(c) for c in np.argwhere(mesh.mesh == rank)[0]]
    A = torch.arange(8 * 12, dtype=torch.float32).reshape(8, 12)
    bad = []
    for src, dst in itertools.product(LAYOUTS, LAYOUTS):
        local = _block(A, src, coord, mesh.topology)
        got = execute(local.clone(), plan(src, dst, 2), mesh)
        if not torch.equal(got, _block(A, dst, coord, mesh.topology)):
            bad.append((src, dst))
    # partial sums along mesh dim 1: the rank with y-coordinate 0 holds the block, the other zeros
    for dst in LAYOUTS:
        src = [0, -1]
        local = _block(A, src, coord, mesh.topology) * (1.0 if coord[1] == 0 else 0.0)
        got = execute(local.clone(), plan(src, dst, 2, partial=[1]), mesh)
        if not torch.equal(got, _block(A, dst, coord, mesh.topology)):
            bad.append(("partial", src, dst))
    # DTensor storage (dygraph auto-parallel): reshard keeps the value, changes the placements
    import paddle_hackathon_amd as paddle
    x = paddle.to_tensor(A.numpy())
    ap.shard_tensor(x, process_mesh=mesh, shard_spec=["x", "y"])
    y = ap.reshard(x, mesh, shard_spec=["y", None])
    full = ap.full_tensor(y).detach()
    local_ok = torch.equal(y._t.to_local(), _block(A, [1, -1], coord, mesh.topology))
    return bad, torch.equal(full, A), local_ok, y.dist_attr["dims_mapping"]


def test_reshard_execution_4_ranks():
    res = run_dist(_worker, 4)
    for bad, full_ok, local_ok, dm in res:
        assert not bad, bad
        assert full_ok and local_ok and dm == [1, -1]
