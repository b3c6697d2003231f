"""``paddle.hub`` (reference: python/paddle/hapi/hub.py): load entrypoints from a repo's
``hubconf.py``. ``source='local'`` loads from a directory; 'github'/'gitee' resolve only
against an already-downloaded copy in the hub cache (no network on the target machines)."""
from __future__ import annotations

import importlib.util
import os
import sys

__all__ = ["list", "help", "load"]

HUB_DIR = os.path.join(os.environ.get("PHA_HOME", os.path.expanduser("~/.cache/paddle_hackathon_amd")), "hub")
_builtin_list = list


def _repo_dir(repo_dir, source, force_reload):
    if source not in ("github", "gitee", "local"):
        raise ValueError(f'Unknown source: "{source}". Allowed values: "github" | "gitee" | "local".')
    if source == "local":
        return repo_dir
    owner_name = repo_dir.split(":")[0].replace("/", "_")
    branch = repo_dir.split(":")[1] if ":" in repo_dir else "main"
    path = os.path.join(HUB_DIR, f"{owner_name}_{branch}")
    if not os.path.isdir(path):
        raise RuntimeError(f"{repo_dir} is not in the local hub cache {HUB_DIR} and downloading is unavailable")
    return path


def _import_hubconf(path):
    f = os.path.join(path, "hubconf.py")
    if not os.path.exists(f):
        raise FileNotFoundError(f"no hubconf.py in {path}")
    sys.path.insert(0, path)
    try:
        spec = importlib.util.spec_from_file_location("hubconf", f)
        m = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(m)
    finally:
        sys.path.remove(path)
    deps = getattr(m, "dependencies", [])
    missing = [d for d in deps if importlib.util.find_spec(d) is None]
    if missing:
        raise RuntimeError(f"Missing dependencies: {', '.join(missing)}")
    return m


def list(repo_dir, source="github", force_reload=False):
    m = _import_hubconf(_repo_dir(repo_dir, source, force_reload))
    return [n for n in dir(m) if callable(getattr(m, n)) and not n.startswith("_")]


def help(repo_dir, model, source="github", force_reload=False):
    m = _import_hubconf(_repo_dir(repo_dir, source, force_reload))
    fn = getattr(m, model, None)
    if fn is None or not callable(fn):
        raise RuntimeError(f"Cannot find callable {model} in hubconf")
    return fn.__doc__


def load(repo_dir, model, source="github", force_reload=False, **kwargs):
    m = _import_hubconf(_repo_dir(repo_dir, source, force_reload))
    fn = getattr(m, model, None)
    if fn is None or not callable(fn):
        raise RuntimeError(f"Cannot find callable {model} in hubconf")
    return fn(**kwargs)
