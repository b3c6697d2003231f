"""Text datasets (reference: python/paddle/text/datasets/*.py).

Sample structures match the reference exactly. ``UCIHousing`` parses the real
``housing.data`` file and ``Imdb`` the real ``aclImdb_v1.tar.gz`` when given; every class
falls back to a deterministic synthetic corpus of the same structure when the file is
absent (no network here). Synthetic size: ``PHA_SYNTHETIC_DATASET_SIZE`` (default 512)."""
from __future__ import annotations

import collections
import os
import re
import tarfile

import numpy as np

from ..io import Dataset

__all__ = ["Conll05st", "Imdb", "Imikolov", "Movielens", "UCIHousing", "WMT14", "WMT16"]


def _n(default=512):
    return int(os.environ.get("PHA_SYNTHETIC_DATASET_SIZE", str(default)))


def _rng(mode, salt):
    return np.random.RandomState((0 if mode == "train" else 1) * 1000 + salt)


class UCIHousing(Dataset):
    """(features float32[13], price float32[1]); features min-max normalised around the mean."""
    FEATURE_NAMES = ["CRIM", "ZN", "INDUS", "CHAS", "NOX", "RM", "AGE", "DIS", "RAD", "TAX", "PTRATIO", "B", "LSTAT"]

    def __init__(self, data_file=None, mode="train", download=True):
        self.mode = mode.lower()
        if data_file and os.path.exists(data_file):
            data = np.fromfile(data_file, sep=" ").reshape(-1, 14)
        else:
            r = _rng("train", 7)
            x = r.rand(506, 13) * 100
            y = x @ r.rand(13) / 10 + r.randn(506)
            data = np.concatenate([x, y[:, None]], 1)
        mx, mn, avg = data.max(0), data.min(0), data.sum(0) / data.shape[0]
        for i in range(13):
            data[:, i] = (data[:, i] - avg[i]) / (mx[i] - mn[i])
        off = int(data.shape[0] * 0.8)
        self.data = (data[:off] if self.mode == "train" else data[off:]).astype("float32")

    def __getitem__(self, idx):
        d = self.data[idx]
        return d[:-1], d[-1:]

    def __len__(self):
        return len(self.data)


class Imdb(Dataset):
    """(word ids int64[L], label int64[1]) — label 0 = positive, 1 = negative (reference order)."""

    def __init__(self, data_file=None, mode="train", cutoff=150, download=True):
        self.mode = mode.lower()
        if data_file and os.path.exists(data_file):
            self.word_idx = self._build_dict(data_file, cutoff)
            self.docs, self.labels = self._load(data_file)
        else:
            r = _rng(self.mode, 3)
            vocab = 5000
            self.word_idx = {f"w{i}": i for i in range(vocab)}
            self.word_idx["<unk>"] = vocab
            n = _n()
            self.labels = r.randint(0, 2, n)
            self.docs = [r.randint(0, vocab, r.randint(20, 200)) + (self.labels[i] * 7 % vocab) for i in range(n)]
            self.docs = [np.clip(d, 0, vocab).astype("int64") for d in self.docs]

    @staticmethod
    def _tok(text):
        return re.sub(r"[^a-z0-9 ]", " ", text.decode("latin-1").lower()).split()

    def _build_dict(self, path, cutoff):
        freq = collections.Counter()
        pat = re.compile(r"aclImdb/train/(pos|neg)/.*\.txt$")
        with tarfile.open(path) as tf:
            for m in tf:
                if pat.match(m.name):
                    freq.update(self._tok(tf.extractfile(m).read()))
        words = sorted([w for w, c in freq.items() if c > cutoff], key=lambda w: (-freq[w], w))
        d = {w: i for i, w in enumerate(words)}
        d["<unk>"] = len(words)
        return d

    def _load(self, path):
        docs, labels = [], []
        unk = self.word_idx["<unk>"]
        with tarfile.open(path) as tf:
            for lab, sub in ((0, "pos"), (1, "neg")):
                pat = re.compile(rf"aclImdb/{self.mode}/{sub}/.*\.txt$")
                for m in tf:
                    if pat.match(m.name):
                        docs.append(np.asarray([self.word_idx.get(w, unk) for w in self._tok(tf.extractfile(m).read())],
                                               dtype="int64"))
                        labels.append(lab)
        return docs, np.asarray(labels)

    def __getitem__(self, idx):
        return self.docs[idx], np.array([self.labels[idx]], dtype="int64")

    def __len__(self):
        return len(self.docs)


class Imikolov(Dataset):
    """PTB language-model data. NGRAM: tuple of ``window_size`` int64 ids; SEQ: (src, trg)."""

    def __init__(self, data_file=None, data_type="NGRAM", window_size=-1, mode="train", min_word_freq=50,
                 download=True):
        self.data_type, self.window_size, self.mode = data_type.upper(), window_size, mode.lower()
        if self.data_type == "NGRAM" and window_size < 1:
            raise ValueError("window_size must be set for NGRAM")
        r = _rng(self.mode, 5)
        vocab = 2000
        self.word_idx = {f"w{i}": i for i in range(vocab)}
        self.word_idx.update({"<s>": vocab, "<e>": vocab + 1, "<unk>": vocab + 2})
        sents = [r.randint(0, vocab, r.randint(5, 30)) for _ in range(_n())]
        self.data = []
        s, e = self.word_idx["<s>"], self.word_idx["<e>"]
        for sent in sents:
            ids = [s] + sent.tolist() + [e]
            if self.data_type == "NGRAM":
                for i in range(window_size, len(ids) + 1):
                    self.data.append(tuple(np.array([w], dtype="int64") for w in ids[i - window_size:i]))
            else:
                self.data.append((np.asarray(ids[:-1], dtype="int64"), np.asarray(ids[1:], dtype="int64")))

    def __getitem__(self, idx):
        return self.data[idx]

    def __len__(self):
        return len(self.data)


class Movielens(Dataset):
    """(user_id, gender, age, job, movie_id, category_ids, title_ids, rating) as int64/float32 arrays."""

    def __init__(self, data_file=None, mode="train", test_ratio=0.1, rand_seed=0, download=True):
        r = np.random.RandomState(rand_seed)
        n = _n(1024)
        self.samples = []
        for _ in range(n):
            self.samples.append((np.array([r.randint(1, 6041)]), np.array([r.randint(0, 2)]),
                                 np.array([r.randint(0, 7)]), np.array([r.randint(0, 21)]),
                                 np.array([r.randint(1, 3953)]), r.randint(0, 18, r.randint(1, 4)),
                                 r.randint(0, 5175, r.randint(1, 8)), np.array([float(r.randint(1, 6))], "float32")))
        is_test = r.rand(n) < test_ratio
        keep = is_test if mode.lower() == "test" else ~is_test
        self.samples = [s for s, k in zip(self.samples, keep) if k]

    def __getitem__(self, idx):
        return tuple(a if a.dtype == np.float32 else a.astype("int64") for a in self.samples[idx])

    def __len__(self):
        return len(self.samples)


class Conll05st(Dataset):
    """SRL: (word, ctx_n2, ctx_n1, ctx_0, ctx_p1, ctx_p2, predicate, mark, label) int64 arrays."""

    def __init__(self, data_file=None, word_dict_file=None, verb_dict_file=None, target_dict_file=None, emb_file=None,
                 download=True):
        r = _rng("test", 11)
        self.word_dict = {f"w{i}": i for i in range(3000)}
        self.predicate_dict = {f"v{i}": i for i in range(300)}
        self.label_dict = {f"l{i}": i for i in range(59)}
        self.samples = []
        for _ in range(_n(256)):
            L = r.randint(5, 40)
            w = r.randint(0, 3000, L)
            ctx = [np.full(L, r.randint(0, 3000)) for _ in range(5)]
            pred = np.full(L, r.randint(0, 300))
            mark = (r.rand(L) < 0.2).astype("int64")
            lab = r.randint(0, 59, L)
            self.samples.append(tuple(a.astype("int64") for a in [w] + ctx + [pred, mark, lab]))

    def get_dict(self):
        return self.word_dict, self.predicate_dict, self.label_dict

    def get_embedding(self):
        return None

    def __getitem__(self, idx):
        return self.samples[idx]

    def __len__(self):
        return len(self.samples)


class _Translation(Dataset):
    START, END, UNK = "<s>", "<e>", "<unk>"

    def _make(self, mode, src_size, trg_size, salt):
        r = _rng(mode, salt)
        self.samples = []
        for _ in range(_n()):
            L = r.randint(3, 50)
            src = np.concatenate([[0], r.randint(3, src_size, L), [1]]).astype("int64")
            trg = r.randint(3, trg_size, r.randint(3, 50))
            self.samples.append((src, np.concatenate([[0], trg]).astype("int64"),
                                 np.concatenate([trg, [1]]).astype("int64")))

    def __getitem__(self, idx):
        return self.samples[idx]

    def __len__(self):
        return len(self.samples)


class WMT14(_Translation):
    """(src_ids, trg_ids, trg_ids_next) with <s>=0, <e>=1, <unk>=2."""

    def __init__(self, data_file=None, mode="train", dict_size=-1, download=True):
        self.dict_size = dict_size if dict_size > 0 else 30000
        self.src_dict = {self.START: 0, self.END: 1, self.UNK: 2}
        self.trg_dict = dict(self.src_dict)
        self._make(mode.lower(), self.dict_size, self.dict_size, 13)

    def get_dict(self, reverse=False):
        return (self.src_dict, self.trg_dict) if not reverse else \
            ({v: k for k, v in self.src_dict.items()}, {v: k for k, v in self.trg_dict.items()})


class WMT16(_Translation):
    def __init__(self, data_file=None, mode="train", src_dict_size=-1, trg_dict_size=-1, lang="en", download=True):
        self.src_dict_size = src_dict_size if src_dict_size > 0 else 10000
        self.trg_dict_size = trg_dict_size if trg_dict_size > 0 else 10000
        self.lang = lang
        self._make(mode.lower(), self.src_dict_size, self.trg_dict_size, 17)

    def get_dict(self, lang, reverse=False):
        d = {self.START: 0, self.END: 1, self.UNK: 2}
        return {v: k for k, v in d.items()} if reverse else d
