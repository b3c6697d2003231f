"""The RCCL ("nccl" backend) code paths on a real MI355X at world size 1 (one GPU per box): the
bucketed DataParallel reducer (native AVG, bf16 buckets, fp32 buckets all-reduced in bf16), the
flat-bucket sharding stages 1-3 with bf16 Linear layers (the collective writes into parameter
storage must refresh the cached transposed weights), the tensor-parallel collectives and the
``init_process_group(device_id=...)`` initialisation. Multi-rank semantics are covered by the gloo
tests in test_distributed.py; these check that every nccl-only branch runs on HIP tensors."""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def nccl_world():
    import paddle_hackathon_amd as paddle
    from paddle_hackathon_amd.parallel import collective as C
    saved = {k: os.environ.get(k) for k in ("MASTER_ADDR", "MASTER_PORT", "RANK", "WORLD_SIZE", "PADDLE_TRAINER_ID",
                                            "PADDLE_TRAINERS_NUM")}
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(_port()), "RANK": "0", "WORLD_SIZE": "1",
                       "PADDLE_TRAINER_ID": "0", "PADDLE_TRAINERS_NUM": "1"})
    g = paddle.distributed.init_parallel_env()
    assert C.get_backend() == "nccl"
    yield g
    C.destroy_process_group()
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


def _bf16_mlp(paddle, seed=0):
    paddle.seed(seed)
    m = paddle.nn.Sequential(paddle.nn.Linear(256, 512), paddle.nn.GELU(), paddle.nn.Linear(512, 256))
    return paddle.amp.decorate(m, level="O2", dtype="bfloat16")


def _batch(step):
    g = torch.Generator(device="cuda")
    g.manual_seed(100 + step)
    x = torch.randn(64, 256, device="cuda", generator=g).bfloat16()
    y = torch.randn(64, 256, device="cuda", generator=g).bfloat16()
    return x, y


def _train(paddle, model, opt, steps=3):
    losses = []
    for s in range(steps):
        x, y = _batch(s)
        out = model(paddle.to_tensor(x))
        loss = ((out - paddle.to_tensor(y)).astype("float32") ** 2).mean()
        loss.backward()
        opt.step()
        opt.clear_grad()
        losses.append(float(loss.item()))
    return losses


def test_collectives_on_hip_tensors(nccl_world):
    import paddle_hackathon_amd as paddle
    import paddle_hackathon_amd.distributed as dist
    x = paddle.to_tensor(torch.arange(8, device="cuda", dtype=torch.float32))
    dist.all_reduce(x)
    dist.all_reduce(x, op=dist.ReduceOp.AVG)
    assert np.allclose(x.numpy(), np.arange(8))
    y = paddle.to_tensor(torch.ones(4, device="cuda", dtype=torch.bfloat16))
    dist.all_reduce(y, op=dist.ReduceOp.MAX)
    lst = []
    dist.all_gather(lst, paddle.to_tensor(torch.full((3,), 2.0, device="cuda")))
    assert len(lst) == 1 and np.allclose(lst[0].numpy(), 2.0)
    rs = paddle.to_tensor(torch.zeros(2, device="cuda"))
    dist.reduce_scatter(rs, [paddle.to_tensor(torch.tensor([1.0, 2.0], device="cuda"))])
    assert np.allclose(rs.numpy(), [1.0, 2.0])
    dist.broadcast(x, src=0)
    dist.barrier()


def test_dataparallel_reducer_nccl_avg_bf16(nccl_world):
    """the reducer's nccl-only branches: ReduceOp.AVG, bf16 buckets, fp32 buckets sent as bf16"""
    import paddle_hackathon_amd as paddle
    from paddle_hackathon_amd.parallel.data_parallel import _Reducer
    ref = _bf16_mlp(paddle)
    m = _bf16_mlp(paddle)
    red = _Reducer(m.parameters(), None, 1 << 16, 1 << 12, False)
    assert red.avg_native and len(red.buckets) > 1
    x, y = _batch(0)
    for model in (ref, m):
        loss = ((model(paddle.to_tensor(x)) - paddle.to_tensor(y)).astype("float32") ** 2).mean()
        loss.backward()
    for p, q in zip(ref.parameters(), m.parameters()):
        assert torch.equal(p._t.grad, q._t.grad)
    # fp32 parameters with a bf16 wire format (strategy.fp16_allreduce)
    paddle.seed(3)
    lin = paddle.nn.Linear(64, 64)
    lin.to(device="gpu")
    red2 = _Reducer(lin.parameters(), None, 1 << 20, 1 << 20, False)
    red2.comm_dtype = torch.bfloat16
    xx = paddle.to_tensor(torch.randn(8, 64, device="cuda"))
    lin(xx).sum().backward()
    g = lin.weight._t.grad.clone()
    assert torch.allclose(g, g.bfloat16().float(), atol=0)   # round-tripped through bf16


@pytest.mark.parametrize("level,extra", [("os", {}), ("os_g", {"buffer_max_size": 1 << 15}),
                                         ("p_g_os", {"segment_size": 1024}),
                                         ("p_g_os", {"segment_size": 1024, "offload": True})])
def test_group_sharded_nccl_bf16_linear_matches_plain(nccl_world, level, extra):
    """sharding on RCCL with bf16 Linear layers (cached transposed weights) for several steps:
    parameters and losses equal plain training (world size 1: the collectives are identities, so
    any stale weight copy or wrong flat-buffer view shows up as a mismatch)"""
    import paddle_hackathon_amd as paddle
    from paddle_hackathon_amd.distributed import group_sharded_parallel
    ref = _bf16_mlp(paddle)
    opt_r = paddle.optimizer.AdamW(1e-2, parameters=ref.parameters(), multi_precision=True,
                                   grad_clip=paddle.nn.ClipGradByGlobalNorm(1.0))
    l_ref = _train(paddle, ref, opt_r)
    m = _bf16_mlp(paddle)
    opt = paddle.optimizer.AdamW(1e-2, parameters=m.parameters(), multi_precision=True,
                                 grad_clip=paddle.nn.ClipGradByGlobalNorm(1.0))
    ms, opt, _ = group_sharded_parallel(m, opt, level, **extra)
    l_sh = _train(paddle, ms, opt)
    np.testing.assert_allclose(l_sh, l_ref, rtol=2e-2, atol=2e-3)
    sd_r, sd_s = ref.state_dict(), ms.state_dict()
    for k in sd_r:
        np.testing.assert_allclose(sd_s[k].astype("float32").numpy(), sd_r[k].astype("float32").numpy(),
                                   rtol=2e-2, atol=2e-2)


def test_tensor_parallel_collectives_nccl(nccl_world):
    import paddle_hackathon_amd as paddle
    from paddle_hackathon_amd.distributed import fleet
    from paddle_hackathon_amd.parallel import mp_layers
    st = fleet.DistributedStrategy()
    st.hybrid_configs = {"dp_degree": 1, "mp_degree": 1, "pp_degree": 1}
    fleet.init(is_collective=True, strategy=st)
    paddle.seed(0)
    col = mp_layers.ColumnParallelLinear(64, 128, has_bias=True, gather_output=True)
    row = mp_layers.RowParallelLinear(128, 64, has_bias=True, input_is_parallel=False)
    x = paddle.to_tensor(torch.randn(4, 64, device="cuda"))
    y = row(col(x))
    y.sum().backward()
    assert y.shape == [4, 64] and col.weight._t.grad is not None
