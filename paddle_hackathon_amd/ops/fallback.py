"""Counter of hot-path fallbacks: every place where a GPU op of the phi hot path (matmul / linear,
conv2d, attention, embedding) leaves the own gfx950 HIP kernels for a library or torch kernel
records it here, with the reason. Tests and the bench assert that the headline models (GPT, BERT,
ResNet-50) record none (``tests/test_kernels_gpu.py::test_headline_paths_have_no_fallbacks``).

``PHA_FALLBACK_LOG=1`` prints each (op, reason) once; ``PHA_STRICT_NATIVE=1`` raises instead.
"""
from __future__ import annotations

import collections
import os
import sys

_counts = collections.Counter()
_lib_counts = collections.Counter()
_seen = set()


def note(op, reason):
    """a GPU ``op`` ran on a non-own kernel because of ``reason``"""
    _counts[op] += 1
    if os.environ.get("PHA_STRICT_NATIVE") == "1":
        raise RuntimeError(f"hot-path fallback: {op} ({reason})")
    if os.environ.get("PHA_FALLBACK_LOG") and (op, reason) not in _seen:
        _seen.add((op, reason))
        print(f"[pha-fallback] {op}: {reason}", file=sys.stderr, flush=True)


def library(op, reason):
    """a GPU ``op`` ran on a vendor-library kernel BY POLICY (the static GEMM policy of ops/gemm.py
    keeps the plain NT forward / dX products on hipBLASLt under PHA_GEMM_IMPL=auto): counted apart
    from the fallbacks so a trace-free run still reports how much of the step left the own kernels.
    PHA_STRICT_LIBRARY=1 raises."""
    _lib_counts[op] += 1
    if os.environ.get("PHA_STRICT_LIBRARY") == "1":
        raise RuntimeError(f"library kernel: {op} ({reason})")
    if os.environ.get("PHA_FALLBACK_LOG") and ("lib", op, reason) not in _seen:
        _seen.add(("lib", op, reason))
        print(f"[pha-library] {op}: {reason}", file=sys.stderr, flush=True)


def library_counts():
    return dict(_lib_counts)


def counts():
    return dict(_counts)


def total():
    return sum(_counts.values())


def reset():
    _counts.clear()
    _lib_counts.clear()
    _seen.clear()
