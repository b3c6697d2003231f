"""Build the native libraries in-tree (no torch headers needed: C ABI + ctypes).

  * ``_C/libpha_kernels.so`` — gfx950 HIP kernels (csrc/kernels/*.hip)
  * ``_C/libpha_runtime.so`` — host C++ runtime (csrc/runtime/*.cpp): data-loader
    ring buffer, gradient bucket planner, host tracer, best-fit arena allocator.
  * ``_C/libpha_infer.so`` — native inference engine with the reference's C API subset
    (csrc/infer, header csrc/infer/pha_infer.h).

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


def _digest(src_files, flags):
    """content hash of the sources + compiler flags + arch (what the library was built from)"""
    import hashlib
    h = hashlib.sha256()
    for s in sorted(src_files):
        h.update(os.path.basename(s).encode())
        with open(s, "rb") as f:
            h.update(f.read())
    # flags name absolute include paths: hash them relative to the package so a tree that moved
    # (the gpurun snapshot lives at another path) still matches its stamps
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    h.update(" ".join(f.replace(root, "<pkg>") for f in flags).encode())
    return h.hexdigest()


def _stale(src_files, target, flags):
    """True unless ``target`` exists and its ``.stamp`` holds the digest of exactly these sources and
    flags. Content-based, not mtime-based: a library that travelled (gpurun snapshot, copy) with
    newer mtimes than edited sources is still rebuilt, and a touched-but-unchanged tree is not."""
    stamp = target + ".stamp"
    if not os.path.exists(target) or not os.path.exists(stamp):
        return True
    with open(stamp) as f:
        return f.read().strip() != _digest(src_files, flags)


def _write_stamp(src_files, target, flags):
    with open(target + ".stamp", "w") as f:
        f.write(_digest(src_files, flags) + "\n")


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
    flags = ["-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC", "-munsafe-fp-atomics",
             "-Wno-unused-result", "-I", os.path.join(CSRC, "kernels")]
    if not force and not _stale(srcs + hdrs + [__file__], target, flags):
        return target
    hipcc = _hipcc()
    objs = []

    def compile_one(src):
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        oflags = flags + _file_flags(src)
        if force or _stale([src] + hdrs, obj, oflags):
            _run([hipcc, "-c", src, "-o", obj] + oflags)
            _write_stamp([src] + hdrs, obj, oflags)
        return obj

    jobs = int(os.environ.get("MAX_JOBS", "8"))
    with cf.ThreadPoolExecutor(max_workers=min(jobs, 16)) as ex:
        objs = list(ex.map(compile_one, srcs))
    _run([hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", target + ".tmp"] + objs)
    os.replace(target + ".tmp", target)
    _write_stamp(srcs + hdrs + [__file__], target, flags)
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
    flags = ["-O3", "-std=c++17", "-Wall", "-shared", "-fPIC", "-pthread"]
    if not force and not _stale(srcs + hdrs + [__file__], target, flags):
        return target
    cxx = shutil.which("g++") or shutil.which("c++")
    _run([cxx] + flags + ["-o", target + ".tmp"] + srcs)
    os.replace(target + ".tmp", target)
    _write_stamp(srcs + hdrs + [__file__], target, flags)
    if verbose:
        print(f"[pha] built {target} from {len(srcs)} C++ sources")
    return target


def build_infer(force=False, verbose=True):
    """``_C/libpha_infer.so`` — the native inference engine + its C API (csrc/infer: host C++ and
    the gfx950 kernels of its device path, linked against the HIP runtime only)"""
    os.makedirs(BUILD, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "infer", "*.cpp")) + glob.glob(os.path.join(CSRC, "infer", "*.hip")))
    hdrs = glob.glob(os.path.join(CSRC, "infer", "*.h"))
    if not srcs:
        return None
    target = os.path.join(OUT, "libpha_infer.so")
    flags = ["-O3", "-std=c++20", f"--offload-arch={ARCH}", "-fPIC", "-shared", "-pthread"]
    if not force and not _stale(srcs + hdrs, target, flags):
        return target
    _run([_hipcc()] + flags + ["-o", target + ".tmp"] + srcs)
    os.replace(target + ".tmp", target)
    _write_stamp(srcs + hdrs, target, flags)
    if verbose:
        print(f"[pha] built {target} (native inference engine)")
    return target


def build_all(force=False, verbose=True):
    return build_kernels(force, verbose), build_runtime(force, verbose), build_infer(force, verbose)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
