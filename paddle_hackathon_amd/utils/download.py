"""Weights download helpers (reference: python/paddle/utils/download.py). There is no network
on the target cluster, so URLs resolve only against a local cache directory
(``$PHA_HOME/weights`` or ``~/.cache/paddle_hackathon_amd/weights``)."""
from __future__ import annotations

import hashlib
import os

WEIGHTS_HOME = os.path.join(os.environ.get("PHA_HOME", os.path.expanduser("~/.cache/paddle_hackathon_amd")), "weights")


def _md5check(path, md5sum=None):
    if md5sum is None:
        return True
    h = hashlib.md5()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest() == md5sum


def get_path_from_url(url, root_dir=WEIGHTS_HOME, md5sum=None, check_exist=True, decompress=True, method="get"):
    path = os.path.join(root_dir, os.path.basename(url.split("?")[0]))
    if os.path.exists(path) and _md5check(path, md5sum):
        return path
    raise FileNotFoundError(f"{path} not found and downloading is unavailable offline (url: {url})")


def get_weights_path_from_url(url, md5sum=None):
    return get_path_from_url(url, WEIGHTS_HOME, md5sum)
