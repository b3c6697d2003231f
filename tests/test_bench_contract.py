"""bench.py launch contract: ``--gpus N`` must never silently run fewer ranks than asked for."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=env,
                          stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=300)


def test_gpus_more_than_visible_fails_loudly():
    import torch
    n = torch.cuda.device_count()
    r = _run(["--gpus", str(max(n + 1, 2)), "--steps", "1", "--warmup", "0"])
    assert r.returncode != 0
    assert "GPU(s) visible" in r.stderr
    assert '"metric"' not in r.stdout


def test_world_size_mismatch_fails():
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0"], {"WORLD_SIZE": "1", "RANK": "0"})
    assert r.returncode == 2
    assert "disagrees" in r.stderr


def test_gpt_micro_batch_steps_down_with_free_memory():
    """the default GPT-3 1.3B micro-batch is 48 only with the HBM for it; an explicit --micro-batch
    and the larger models are left alone"""
    import importlib.util
    import types
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)

    def fake_torch(free_gb):
        cuda = types.SimpleNamespace(mem_get_info=lambda: (free_gb * 2 ** 30, 288 * 2 ** 30),
                                     device_count=lambda: 1)
        return types.SimpleNamespace(cuda=cuda)

    def args(mb=None, model="gpt3-1.3b", tp=1, pp=1, sharding_stage=0, recompute=False):
        return types.SimpleNamespace(micro_batch=mb, model=model, tp=tp, pp=pp, sharding_stage=sharding_stage,
                                     recompute=recompute)
    assert bench._gpt_micro_batch(args(), fake_torch(287), 1, 0) == 48
    assert bench._gpt_micro_batch(args(), fake_torch(180), 1, 0) == 32
    assert bench._gpt_micro_batch(args(), fake_torch(100), 1, 0) == 16
    assert bench._gpt_micro_batch(args(mb=12), fake_torch(20), 1, 0) == 12
    assert bench._gpt_micro_batch(args(model="gpt3-13b"), fake_torch(287), 1, 0) == 2
    # the free-memory thresholds were measured for the plain DP layout: other layouts take 16
    assert bench._gpt_micro_batch(args(tp=4), fake_torch(287), 1, 0) == 16
    assert bench._gpt_micro_batch(args(pp=2, sharding_stage=3, recompute=True), fake_torch(287), 1, 0) == 16
