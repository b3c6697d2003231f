"""bench.py's GPT construction path (models/gpt_train.py GPTTrainer) for every fleet layout the
benchmark can run — dp2, dp2 x tp2, pp2 x sharding2 (stage 1 / 2 / 3) — on gloo ranks at tiny size:
the per-step loss averaged over the data ranks equals single-process training on the whole batch
(reference test pattern: hybrid_parallel_* tests vs a single-card model with the same seed)."""
import numpy as np
import pytest

from dist_helper import run_dist

pytestmark = [pytest.mark.dist, pytest.mark.timeout(600)]

STEPS, B, S = 3, 2, 16
CFG = {"hidden_dropout": 0.0, "attention_dropout": 0.0}


def _state():
    import paddle_hackathon_amd as paddle
    from paddle_hackathon_amd.models import gpt_config, GPTForPretraining
    paddle.set_device("cpu")
    paddle.seed(17)
    m = GPTForPretraining(gpt_config("gpt-tiny", **CFG))
    return {k: v.numpy() for k, v in m.state_dict().items()}


def _ids(n_rows):
    return np.random.RandomState(8).randint(0, 512, (n_rows, S + 1)).astype("int64")


def _tp_slice(state, model, rank, tp):
    out = {}
    params = dict(model.named_parameters())
    for name, v in state.items():
        p = params.get(name)
        if p is None or tuple(p.shape) == v.shape:
            out[name] = v
            continue
        d = [i for i in range(v.ndim) if v.shape[i] != p.shape[i]][0]
        out[name] = np.ascontiguousarray(np.split(v, tp, axis=d)[rank % tp])
    return out


def _run(rank, world, layout_kw, state):
    import paddle_hackathon_amd as paddle
    from paddle_hackathon_amd.models.gpt_train import GPTTrainer, Layout
    lo = Layout(world=world, **layout_kw)
    st = state
    if lo.tp > 1:   # each TP rank loads its slice of the full state
        from paddle_hackathon_amd.models import gpt_config, GPTForPretraining
        from paddle_hackathon_amd.distributed import fleet
        tr = GPTTrainer("gpt-tiny", lo, rank, lr=1e-2, amp=False, cfg_overrides=CFG)
        hcg = fleet.get_hybrid_communicate_group()
        sliced = _tp_slice(state, tr.inner, hcg.get_model_parallel_rank(), lo.tp)
        tr.inner.set_state_dict({k: paddle.to_tensor(v) for k, v in sliced.items()})
    else:
        tr = GPTTrainer("gpt-tiny", lo, rank, lr=1e-2, amp=False, cfg_overrides=CFG, state=st)
    ids = _ids(B * lo.data_ranks)
    d = tr.data_rank()
    mine = ids[d * B:(d + 1) * B]
    inp, lab = paddle.to_tensor(mine[:, :-1]), paddle.to_tensor(mine[:, 1:])
    losses = [float(tr.step(inp, lab).numpy()) for _ in range(STEPS)]
    return {"losses": losses, "data_rank": d, "name": lo.name()}


def _reference(state, data_ranks):
    import paddle_hackathon_amd as paddle
    from paddle_hackathon_amd.models.gpt_train import GPTTrainer, Layout
    paddle.set_device("cpu")
    tr = GPTTrainer("gpt-tiny", Layout(world=1), 0, lr=1e-2, amp=False, cfg_overrides=CFG, state=state)
    ids = _ids(B * data_ranks)
    inp, lab = paddle.to_tensor(ids[:, :-1]), paddle.to_tensor(ids[:, 1:])
    return [float(tr.step(inp, lab).numpy()) for _ in range(STEPS)]


@pytest.mark.parametrize("world,layout", [
    (2, {}),                                                          # dp2
    (4, {"tp": 2}),                                                   # dp2 x tp2
    (4, {"pp": 2, "sharding_stage": 1, "micro_batches": 2}),          # pp2 x sharding2 (os)
    (4, {"pp": 2, "sharding_stage": 2, "micro_batches": 2}),          # pp2 x sharding2 (os_g)
    (4, {"pp": 2, "sharding_stage": 3, "micro_batches": 2}),          # pp2 x sharding2 (p_g_os)
], ids=["dp2", "dp2_tp2", "pp2_sharding2_s1", "pp2_sharding2_s2", "pp2_sharding2_s3"])
def test_layout_matches_single_process(world, layout):
    state = _state()
    res = run_dist(_run, world, args=(layout, state))
    data_ranks = max(r["data_rank"] for r in res) + 1
    ref = _reference(state, data_ranks)
    by_d = {}
    for r in res:
        by_d.setdefault(r["data_rank"], []).append(r["losses"])
    for d, ls in by_d.items():   # peers of one data rank (TP / PP) agree
        for l in ls[1:]:
            np.testing.assert_allclose(l, ls[0], rtol=1e-5)
    mean = np.mean([by_d[d][0] for d in sorted(by_d)], axis=0)
    np.testing.assert_allclose(mean, ref, rtol=2e-4, atol=2e-5)
