"""Build the native libraries in-tree (no torch headers needed: C ABI + ctypes).

  * ``_C/libpha_kernels.so`` — gfx950 HIP kernels (csrc/kernels/*.hip)
  * ``_C/libpha_runtime.so`` — host C++ runtime (csrc/runtime/*.cpp): data-loader
    ring buffer, gradient bucket planner, host tracer, best-fit arena allocator.

Usage: ``python -m paddle_hackathon_amd.ops.build [--force]``.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(PKG, "csrc")
OUT = os.path.join(PKG, "_C")
BUILD = os.path.join(OUT, "build")
ARCH = os.environ.get("PHA_OFFLOAD_ARCH", "gfx950")


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def _newer(src_files, target):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in src_files)


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n" + " ".join(cmd) + "\n" + r.stdout)
    return r.stdout


def _file_flags(src):
    """Per-source extra compiler flags from a ``// pha-build-flags: ...`` line in its header."""
    with open(src) as f:
        for _, line in zip(range(40), f):
            if line.startswith("// pha-build-flags:"):
                return line.split(":", 1)[1].split()
    return []


def build_kernels(force=False, verbose=True):
    os.makedirs(BUILD, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    hdrs = glob.glob(os.path.join(CSRC, "kernels", "*.h"))
    target = os.path.join(OUT, "libpha_kernels.so")
    if not force and not _newer(srcs + hdrs + [__file__], target):
        return target
    hipcc = _hipcc()
    flags = ["-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC", "-munsafe-fp-atomics",
             "-Wno-unused-result", "-I", os.path.join(CSRC, "kernels")]
    objs = []

    def compile_one(src):
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        if force or _newer([src] + hdrs, obj):
            _run([hipcc, "-c", src, "-o", obj] + flags + _file_flags(src))
        return obj

    jobs = int(os.environ.get("MAX_JOBS", "8"))
    with cf.ThreadPoolExecutor(max_workers=min(jobs, 16)) as ex:
        objs = list(ex.map(compile_one, srcs))
    _run([hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", target + ".tmp"] + objs)
    os.replace(target + ".tmp", target)
    if verbose:
        print(f"[pha] built {target} from {len(srcs)} HIP sources for {ARCH}")
    return target


def build_runtime(force=False, verbose=True):
    os.makedirs(BUILD, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    hdrs = glob.glob(os.path.join(CSRC, "runtime", "*.h"))
    if not srcs:
        return None
    target = os.path.join(OUT, "libpha_runtime.so")
    if not force and not _newer(srcs + hdrs + [__file__], target):
        return target
    cxx = shutil.which("g++") or shutil.which("c++")
    _run([cxx, "-O3", "-std=c++17", "-Wall", "-shared", "-fPIC", "-pthread", "-o", target + ".tmp"] + srcs)
    os.replace(target + ".tmp", target)
    if verbose:
        print(f"[pha] built {target} from {len(srcs)} C++ sources")
    return target


def build_all(force=False, verbose=True):
    return build_kernels(force, verbose), build_runtime(force, verbose)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
