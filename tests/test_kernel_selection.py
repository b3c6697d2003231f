"""Kernel selection is static and deterministic (CPU): the GEMM per-layout policy and the conv tile
table (ops/conv_gemm.py) — no timing on first use unless the reference's opt-in kernel autotune
is enabled."""
import torch


def test_conv_tuning_table_loads_and_is_used():
    from paddle_hackathon_amd.ops import conv_gemm as cg
    tab = cg._table()
    assert len(tab) >= 60
    for k, v in tab.items():
        kind = k.split("|")[0]
        assert kind in ("conv", "wgrad"), k
        assert (isinstance(v, list) and len(v) == 2 and all(isinstance(a, int) for a in v)) or isinstance(v, int), v
    key_s = next(k for k in tab if k.startswith("conv|"))
    parts = key_s.split("|")
    key = (parts[0], torch.bfloat16) + tuple(int(p) for p in parts[2:])
    assert cg._kstr(key) == key_s
    cg._tuned.pop(key, None)
    assert cg._lookup(key) == tuple(tab[key_s])


def test_conv_timing_autotune_is_opt_in(monkeypatch):
    from paddle_hackathon_amd.ops import conv_gemm as cg
    from paddle_hackathon_amd.incubate import autotune
    monkeypatch.delenv("PHA_G256_AUTOTUNE", raising=False)
    cg._timing_on[0] = None
    assert not cg._timing()
    calls = []
    assert cg._autotune(("conv", "unknown-shape"), lambda *a: calls.append(a)) == (-1, 0)
    assert not calls, "no timing runs without opt-in"
    autotune.set_config({"kernel": {"enable": True}})
    try:
        assert cg._timing()
    finally:
        autotune.set_config({"kernel": {"enable": False}})
        cg._timing_on[0] = None
    assert not cg._timing()


def test_tn_pick_carries_split_factor(monkeypatch):
    """a weight-gradient table entry [tile, splits] fixes the split-K factor too; a bare tile keeps
    the formula's splits"""
    from paddle_hackathon_amd.ops import conv_gemm as cg
    key = ("wgrad", "synthetic-shape")
    monkeypatch.setattr(cg, "_tn_ws", lambda sp, M, N, dev: None)
    monkeypatch.setattr(cg, "_num_cus", lambda dev: 256)
    calls = []
    monkeypatch.setitem(cg._tuned, key, (3, 48))
    cg._run_tn(key, 128, 1152, 200704, "cpu", lambda t, sp, ws: calls.append((t, sp)))
    monkeypatch.setitem(cg._tuned, key, 3)
    cg._run_tn(key, 128, 1152, 200704, "cpu", lambda t, sp, ws: calls.append((t, sp)))
    assert calls == [(3, 48), (3, cg._tn_splits(128, 1152, 200704, 3, "cpu"))]


def test_gemm_policy_is_static(monkeypatch):
    from paddle_hackathon_amd.ops import gemm as G
    monkeypatch.setenv("PHA_GEMM_IMPL", "auto")
    assert G._AUTO_OWN == ("tn", "nn")
    cpu = torch.zeros(8, 64, dtype=torch.bfloat16)
    assert not G._own_ok("nt", cpu, cpu)     # library NT under auto, own never on CPU tensors
    monkeypatch.setenv("PHA_GEMM_IMPL", "library")
    assert not G._own_ok("tn", cpu, cpu)
