"""Build an A/B variant of one kernel source: compile it with extra -D flags and link it with the
other in-tree objects into paddle_hackathon_amd/_C/libpha_kernels_<name>.so (load it with
PHA_KERNELS_LIB=libpha_kernels_<name>.so). usage: build_variant.py NAME SOURCE.hip [-DFOO=1 ...]"""
import glob
import os
import subprocess
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from paddle_hackathon_amd.ops import build  # noqa: E402

name, src, defs = sys.argv[1], sys.argv[2], sys.argv[3:]
build.build_kernels(verbose=False)
kdir = os.path.join(build.CSRC, "kernels")
src_path = os.path.join(kdir, src)
obj = f"/tmp/variant_{name}_{src}.o"
flags = ["-O3", "-std=c++17", f"--offload-arch={build.ARCH}", "-fPIC", "-munsafe-fp-atomics", "-Wno-unused-result",
         "-Wno-inline-asm", "-I", kdir] + build._file_flags(src_path) + defs
subprocess.check_call([build._hipcc(), "-c", src_path, "-o", obj] + flags)
objs = [o for o in glob.glob(os.path.join(build.BUILD, "*.hip.o")) if os.path.basename(o) != src + ".o"] + [obj]
out = os.path.join(build.OUT, f"libpha_kernels_{name}.so")
subprocess.check_call([build._hipcc(), "-shared", "-fPIC", f"--offload-arch={build.ARCH}", "-o", out] + objs)
print("built", out)
