"""Vision datasets (reference: python/paddle/vision/datasets/*). No network here: each
dataset reads the standard on-disk format from ``data_file`` / ``image_path`` when given, and
otherwise (``download=True`` with no file) yields a deterministic synthetic set of the right
shapes so pipelines and tests run offline."""
from __future__ import annotations

import gzip
import os
import pickle
import struct
import tarfile

import numpy as np

from ..io import Dataset

__all__ = ["MNIST", "FashionMNIST", "Cifar10", "Cifar100", "Flowers", "VOC2012", "DatasetFolder", "ImageFolder",
           "SyntheticImages"]

IMG_EXTENSIONS = (".jpg", ".jpeg", ".png", ".ppm", ".bmp", ".pgm", ".tif", ".tiff", ".webp")


class SyntheticImages(Dataset):
    def __init__(self, n, shape, num_classes, dtype="float32", seed=0, transform=None):
        rng = np.random.RandomState(seed)
        self.images = (rng.rand(n, *shape) * 255).astype("uint8")
        self.labels = rng.randint(0, num_classes, (n, 1)).astype("int64")
        self.transform, self.dtype = transform, dtype

    def __getitem__(self, i):
        img = self.images[i]
        if self.transform is not None:
            img = self.transform(img)
        else:
            img = img.astype(self.dtype)
        return img, self.labels[i]

    def __len__(self):
        return len(self.images)


class _RestrictedUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        if module.startswith("numpy") or (module, name) in {("builtins", "dict"), ("builtins", "list")}:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"refusing {module}.{name}")


class MNIST(Dataset):
    NAME = "mnist"

    def __init__(self, image_path=None, label_path=None, mode="train", transform=None, download=True, backend=None):
        self.mode, self.transform, self.backend = mode.lower(), transform, backend or "cv2"
        if image_path and label_path and os.path.exists(image_path):
            self.images, self.labels = self._parse(image_path, label_path)
        else:
            n = 60000 if self.mode == "train" else 10000
            n = min(n, int(os.environ.get("PHA_SYNTHETIC_DATASET_SIZE", "2048")))
            syn = SyntheticImages(n, (28, 28), 10, seed=0 if self.mode == "train" else 1)
            self.images, self.labels = syn.images, syn.labels

    @staticmethod
    def _open(p):
        return gzip.open(p, "rb") if p.endswith(".gz") else open(p, "rb")

    def _parse(self, ip, lp):
        with self._open(ip) as f:
            _, n, r, c = struct.unpack(">IIII", f.read(16))
            imgs = np.frombuffer(f.read(), dtype=np.uint8).reshape(n, r, c)
        with self._open(lp) as f:
            struct.unpack(">II", f.read(8))
            labs = np.frombuffer(f.read(), dtype=np.uint8).astype("int64").reshape(-1, 1)
        return imgs, labs

    def __getitem__(self, idx):
        img, label = self.images[idx], self.labels[idx]
        if self.transform is not None:
            img = self.transform(img if self.backend != "pil" else __import__("PIL.Image").Image.fromarray(img))
        else:
            img = img.astype("float32")[None] / 255.0
        return img, label

    def __len__(self):
        return len(self.labels)


class FashionMNIST(MNIST):
    NAME = "fashion-mnist"


class Cifar10(Dataset):
    _NUM = 10

    def __init__(self, data_file=None, mode="train", transform=None, download=True, backend=None):
        self.mode, self.transform = mode.lower(), transform
        self.data = []
        if data_file and os.path.exists(data_file):
            with tarfile.open(data_file) as tf:
                key = "data_batch" if self.mode == "train" else "test_batch"
                for m in tf.getmembers():
                    if key in m.name or (self._NUM == 100 and (self.mode in m.name)):
                        d = _RestrictedUnpickler(tf.extractfile(m), encoding="bytes").load()
                        labels = d.get(b"labels", d.get(b"fine_labels"))
                        for img, lab in zip(d[b"data"], labels):
                            self.data.append((np.asarray(img, np.uint8).reshape(3, 32, 32).transpose(1, 2, 0), int(lab)))
        else:
            n = min(50000 if self.mode == "train" else 10000, int(os.environ.get("PHA_SYNTHETIC_DATASET_SIZE", "2048")))
            syn = SyntheticImages(n, (32, 32, 3), self._NUM, seed=2)
            self.data = [(syn.images[i], int(syn.labels[i, 0])) for i in range(n)]

    def __getitem__(self, idx):
        img, label = self.data[idx]
        if self.transform is not None:
            img = self.transform(img)
        else:
            img = img.astype("float32").transpose(2, 0, 1) / 255.0
        return img, np.array([label], dtype="int64")

    def __len__(self):
        return len(self.data)


class Cifar100(Cifar10):
    _NUM = 100


class Flowers(Dataset):
    def __init__(self, data_file=None, label_file=None, setid_file=None, mode="train", transform=None, download=True,
                 backend=None):
        n = int(os.environ.get("PHA_SYNTHETIC_DATASET_SIZE", "256"))
        syn = SyntheticImages(n, (64, 64, 3), 102, seed=3)
        self.images, self.labels, self.transform = syn.images, syn.labels, transform

    def __getitem__(self, idx):
        img = self.images[idx]
        img = self.transform(img) if self.transform else img.astype("float32").transpose(2, 0, 1) / 255.0
        return img, self.labels[idx]

    def __len__(self):
        return len(self.images)


class VOC2012(Dataset):
    def __init__(self, data_file=None, mode="train", transform=None, download=True, backend=None):
        n = int(os.environ.get("PHA_SYNTHETIC_DATASET_SIZE", "64"))
        rng = np.random.RandomState(4)
        self.images = (rng.rand(n, 64, 64, 3) * 255).astype("uint8")
        self.labels = rng.randint(0, 21, (n, 64, 64)).astype("uint8")
        self.transform = transform

    def __getitem__(self, idx):
        img = self.images[idx]
        img = self.transform(img) if self.transform else img.astype("float32")
        return img, self.labels[idx]

    def __len__(self):
        return len(self.images)


def _default_loader(path):
    from PIL import Image
    with open(path, "rb") as f:
        return np.asarray(Image.open(f).convert("RGB"))


class DatasetFolder(Dataset):
    def __init__(self, root, loader=None, extensions=None, transform=None, is_valid_file=None):
        self.root, self.loader, self.transform = root, loader or _default_loader, transform
        exts = tuple(extensions) if extensions else IMG_EXTENSIONS
        classes = sorted(d.name for d in os.scandir(root) if d.is_dir())
        self.classes = classes
        self.class_to_idx = {c: i for i, c in enumerate(classes)}
        samples = []
        for c in classes:
            for dp, _, fns in sorted(os.walk(os.path.join(root, c))):
                for fn in sorted(fns):
                    p = os.path.join(dp, fn)
                    ok = is_valid_file(p) if is_valid_file else fn.lower().endswith(exts)
                    if ok:
                        samples.append((p, self.class_to_idx[c]))
        self.samples = samples
        self.targets = [s[1] for s in samples]

    def __getitem__(self, idx):
        path, target = self.samples[idx]
        sample = self.loader(path)
        if self.transform is not None:
            sample = self.transform(sample)
        return sample, target

    def __len__(self):
        return len(self.samples)


class ImageFolder(Dataset):
    def __init__(self, root, loader=None, extensions=None, transform=None, is_valid_file=None):
        self.root, self.loader, self.transform = root, loader or _default_loader, transform
        exts = tuple(extensions) if extensions else IMG_EXTENSIONS
        self.samples = []
        for dp, _, fns in sorted(os.walk(root)):
            for fn in sorted(fns):
                p = os.path.join(dp, fn)
                if (is_valid_file(p) if is_valid_file else fn.lower().endswith(exts)):
                    self.samples.append(p)

    def __getitem__(self, idx):
        s = self.loader(self.samples[idx])
        if self.transform is not None:
            s = self.transform(s)
        return [s]

    def __len__(self):
        return len(self.samples)
