"""DBoW2 vocabulary in the ORBvoc.txt layout.

Text format (TemplatedVocabulary::loadFromTextFile / saveToTextFile):
    line 0:  k L scoring weighting
    line i:  parent is_leaf d0 ... d31 weight      (node i, i >= 1; node 0 is the root)
Children keep file order. Word ids are numbered in order of leaf appearance. ORB-SLAM3 uses
k=10, L=6, TF_IDF weighting and L1_NORM scoring. ORBvoc.txt itself is not in the reference
(R:.gitignore), so tests and benchmarks use `Vocabulary.synthetic`. That is a deterministic
k-ary tree: random node descriptors, each child a bit-flip perturbation of its parent, so that
similar descriptors descend the same path, with IDF-like positive leaf weights.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

TF_IDF, L1_NORM = 0, 0


@dataclass
class Vocabulary:
    k: int
    L: int
    scoring: int
    weighting: int
    parent: np.ndarray     # [N] int32 (parent[0] = -1: root)
    is_leaf: np.ndarray    # [N] uint8
    desc: np.ndarray       # [N, 32] uint8 (row 0 unused)
    weight: np.ndarray     # [N] float64

    @property
    def n_nodes(self) -> int:
        return int(self.parent.shape[0])

    # ---- derived tables (CSR children in file order, word ids in leaf order) ----
    def csr(self):
        N = self.n_nodes
        par = self.parent[1:]
        n_child = np.bincount(par, minlength=N).astype(np.int32)
        first = np.zeros(N, np.int32)
        first[1:] = np.cumsum(n_child)[:-1]
        order = np.argsort(par, kind="stable").astype(np.int32) + 1   # children grouped by parent, file order
        word = np.full(N, -1, np.int32)
        leaves = np.nonzero(self.is_leaf)[0]
        word[leaves] = np.arange(len(leaves), dtype=np.int32)
        return first, n_child, order, word

    # ---- ORBvoc.txt ----
    def save_text(self, path: str):
        with open(path, "w") as f:
            f.write(f"{self.k} {self.L} {self.scoring} {self.weighting}\n")
            for i in range(1, self.n_nodes):
                d = " ".join(str(int(v)) for v in self.desc[i])
                f.write(f"{int(self.parent[i])} {int(self.is_leaf[i])} {d} {float(self.weight[i])!r}\n")

    @staticmethod
    def load_text(path: str) -> "Vocabulary":
        with open(path) as f:
            k, L, scoring, weighting = (int(v) for v in f.readline().split())
            rows = [line.split() for line in f if line.strip()]
        N = len(rows) + 1
        parent = np.full(N, -1, np.int32)
        is_leaf = np.zeros(N, np.uint8)
        desc = np.zeros((N, 32), np.uint8)
        weight = np.zeros(N, np.float64)
        for i, r in enumerate(rows, start=1):
            parent[i] = int(r[0])
            is_leaf[i] = int(r[1])
            desc[i] = np.array([int(v) for v in r[2:34]], np.uint8)
            weight[i] = float(r[34])
        return Vocabulary(k, L, scoring, weighting, parent, is_leaf, desc, weight)

    # ---- synthetic vocabulary (deterministic) ----
    @staticmethod
    def synthetic(k: int = 10, L: int = 6, seed: int = 0) -> "Vocabulary":
        rng = np.random.Generator(np.random.PCG64(seed))
        sizes = [k ** l for l in range(L + 1)]
        N = sum(sizes)
        parent = np.full(N, -1, np.int32)
        desc = np.zeros((N, 32), np.uint8)
        start = 1
        prev = np.array([0])
        prev_desc = rng.integers(0, 256, (1, 32), dtype=np.uint8)
        for l in range(1, L + 1):
            n = sizes[l]
            par = np.repeat(prev, k)
            parent[start:start + n] = par
            base = np.repeat(prev_desc, k, axis=0)
            if l == 1:
                d = rng.integers(0, 256, (n, 32), dtype=np.uint8)
            else:   # children = parent's descriptor with ~1/8 of its bits flipped (AND of 3 random masks)
                m = rng.integers(0, 256, base.shape, dtype=np.uint8)
                m &= rng.integers(0, 256, base.shape, dtype=np.uint8)
                m &= rng.integers(0, 256, base.shape, dtype=np.uint8)
                d = base ^ m
            desc[start:start + n] = d
            prev = np.arange(start, start + n)
            prev_desc = d
            start += n
        is_leaf = np.zeros(N, np.uint8)
        is_leaf[N - sizes[L]:] = 1
        weight = np.zeros(N, np.float64)
        weight[N - sizes[L]:] = rng.uniform(0.5, 8.0, sizes[L])   # idf = log(N / n_i) > 0
        return Vocabulary(k, L, L1_NORM, TF_IDF, parent, is_leaf, desc, weight)


def bow_vector(word: np.ndarray, weight: np.ndarray):
    """BowVector (TF_IDF + L1_NORM) from per-feature (word, weight): sorted word ids, values."""
    m = weight > 0
    w, inv = np.unique(word[m], return_inverse=True)
    v = np.zeros(len(w))
    np.add.at(v, inv, weight[m])                 # per word, in feature order (BowVector::addWeight)
    s = float(np.cumsum(np.abs(v))[-1]) if len(v) else 0.0   # sequential, as BowVector::normalize(L1)
    return w.astype(np.int32), (v / s if s > 0 else v)


def feature_vector(node: np.ndarray, weight: np.ndarray):
    """FeatureVector: {node id: ascending feature indices} of the features with weight > 0."""
    fv = {}
    for i in np.nonzero(weight > 0)[0]:
        fv.setdefault(int(node[i]), []).append(int(i))
    return dict(sorted(fv.items()))
