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
