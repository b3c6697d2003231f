"""fleet.utils (reference: python/paddle/distributed/fleet/utils/__init__.py)."""
from ...recompute import recompute, recompute_sequential  # noqa: F401
from . import hybrid_parallel_util, hybrid_parallel_inference  # noqa: F401
from .hybrid_parallel_inference import HybridParallelInferenceHelper  # noqa: F401


class LocalFS:
    """Local filesystem helper (reference: fleet/utils/fs.py:LocalFS)."""

    def ls_dir(self, fs_path):
        import os
        if not os.path.exists(fs_path):
            return [], []
        dirs, files = [], []
        for f in os.listdir(fs_path):
            (dirs if os.path.isdir(os.path.join(fs_path, f)) else files).append(f)
        return dirs, files

    def mkdirs(self, fs_path):
        import os
        os.makedirs(fs_path, exist_ok=True)

    def is_exist(self, fs_path):
        import os
        return os.path.exists(fs_path)

    def is_dir(self, fs_path):
        import os
        return os.path.isdir(fs_path)

    def is_file(self, fs_path):
        import os
        return os.path.isfile(fs_path)

    def delete(self, fs_path):
        import os
        import shutil
        if os.path.isdir(fs_path):
            shutil.rmtree(fs_path)
        elif os.path.exists(fs_path):
            os.remove(fs_path)

    def rename(self, src, dst):
        import os
        os.rename(src, dst)

    def touch(self, fs_path, exist_ok=True):
        open(fs_path, "a").close()


class HDFSClient(LocalFS):
    def __init__(self, hadoop_home=None, configs=None, *a, **k):
        raise RuntimeError("HDFS is not available in this environment")
