"""Legacy reader-creator datasets (reference: python/paddle/dataset/*.py): each module has
``train()`` / ``test()`` returning a no-arg generator function of samples, backed by the
``paddle.vision.datasets`` / ``paddle.text.datasets`` classes (synthetic offline)."""
from __future__ import annotations

import sys
import types

import numpy as np

__all__ = ["mnist", "cifar", "uci_housing", "imdb", "imikolov", "movielens", "conll05", "wmt14", "wmt16", "flowers",
           "voc2012", "common", "image"]


def _reader(make, convert):
    def creator():
        ds = make()
        for i in range(len(ds)):
            yield convert(ds[i])
    return creator


def _mod(name, **fns):
    m = types.ModuleType(f"{__name__}.{name}")
    m.__dict__.update(fns)
    sys.modules[m.__name__] = m
    return m


def _img_flat(s):
    img, lab = s
    a = np.asarray(img, dtype="float32").reshape(-1)
    if a.max() > 1.0:
        a = a / 255.0
    return a * 2.0 - 1.0, int(np.asarray(lab).reshape(-1)[0])


def _vision(cls, mode, **kw):
    from ..vision import datasets as V
    return lambda: getattr(V, cls)(mode=mode, **kw)


def _text(cls, **kw):
    from ..text import datasets as T
    return lambda: getattr(T, cls)(**kw)


mnist = _mod("mnist", train=lambda: _reader(_vision("MNIST", "train"), _img_flat),
             test=lambda: _reader(_vision("MNIST", "test"), _img_flat))
cifar = _mod("cifar", train10=lambda cycle=False: _reader(_vision("Cifar10", "train"), _img_flat),
             test10=lambda cycle=False: _reader(_vision("Cifar10", "test"), _img_flat),
             train100=lambda: _reader(_vision("Cifar100", "train"), _img_flat),
             test100=lambda: _reader(_vision("Cifar100", "test"), _img_flat))
flowers = _mod("flowers", train=lambda mapper=None, buffered_size=1024, use_xmap=True, cycle=False:
               _reader(_vision("Flowers", "train"), _img_flat),
               test=lambda mapper=None, buffered_size=1024, use_xmap=True, cycle=False:
               _reader(_vision("Flowers", "test"), _img_flat),
               valid=lambda mapper=None, buffered_size=1024, use_xmap=True:
               _reader(_vision("Flowers", "valid"), _img_flat))
voc2012 = _mod("voc2012", train=lambda: _reader(_vision("VOC2012", "train"), tuple),
               test=lambda: _reader(_vision("VOC2012", "test"), tuple),
               val=lambda: _reader(_vision("VOC2012", "valid"), tuple))
uci_housing = _mod("uci_housing", train=lambda: _reader(_text("UCIHousing", mode="train"), tuple),
                   test=lambda: _reader(_text("UCIHousing", mode="test"), tuple),
                   feature_names=["CRIM", "ZN", "INDUS", "CHAS", "NOX", "RM", "AGE", "DIS", "RAD", "TAX", "PTRATIO",
                                  "B", "LSTAT"])
imdb = _mod("imdb", word_dict=lambda cutoff=150: _text("Imdb", mode="train", cutoff=cutoff)().word_idx,
            train=lambda word_idx=None: _reader(_text("Imdb", mode="train"),
                                                lambda s: (s[0].tolist(), int(s[1][0]))),
            test=lambda word_idx=None: _reader(_text("Imdb", mode="test"), lambda s: (s[0].tolist(), int(s[1][0]))))
imikolov = _mod("imikolov", build_dict=lambda min_word_freq=50: _text("Imikolov", window_size=2)().word_idx,
                train=lambda word_idx=None, n=5, data_type=1: _reader(
                    _text("Imikolov", window_size=n, mode="train"), lambda s: tuple(int(a[0]) for a in s)),
                test=lambda word_idx=None, n=5, data_type=1: _reader(
                    _text("Imikolov", window_size=n, mode="test"), lambda s: tuple(int(a[0]) for a in s)))
movielens = _mod("movielens", train=lambda: _reader(_text("Movielens", mode="train"), tuple),
                 test=lambda: _reader(_text("Movielens", mode="test"), tuple))
conll05 = _mod("conll05", test=lambda: _reader(_text("Conll05st"), tuple),
               get_dict=lambda: _text("Conll05st")().get_dict())
wmt14 = _mod("wmt14", train=lambda dict_size: _reader(_text("WMT14", mode="train", dict_size=dict_size), tuple),
             test=lambda dict_size: _reader(_text("WMT14", mode="test", dict_size=dict_size), tuple))
wmt16 = _mod("wmt16", train=lambda src_dict_size, trg_dict_size, src_lang="en": _reader(
    _text("WMT16", mode="train", src_dict_size=src_dict_size, trg_dict_size=trg_dict_size, lang=src_lang), tuple),
             test=lambda src_dict_size, trg_dict_size, src_lang="en": _reader(
    _text("WMT16", mode="test", src_dict_size=src_dict_size, trg_dict_size=trg_dict_size, lang=src_lang), tuple))
common = _mod("common", DATA_HOME=__import__("os").path.expanduser("~/.cache/paddle_hackathon_amd/dataset"),
              md5file=lambda fname: __import__("hashlib").md5(open(fname, "rb").read()).hexdigest())


def _img_load(file, is_color=True):
    from PIL import Image
    im = Image.open(file)
    return np.asarray(im.convert("RGB" if is_color else "L"))


image = _mod("image", load_image=_img_load,
             to_chw=lambda im, order=(2, 0, 1): im.transpose(order),
             center_crop=lambda im, size, is_color=True: im[(im.shape[0] - size) // 2:(im.shape[0] - size) // 2 + size,
                                                            (im.shape[1] - size) // 2:(im.shape[1] - size) // 2 + size],
             left_right_flip=lambda im, is_color=True: im[:, ::-1])
