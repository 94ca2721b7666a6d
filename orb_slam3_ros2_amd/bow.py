"""ORBVocabulary mirror (Thirdparty/DBoW2 TemplatedVocabulary<FORB> as ORB_SLAM3 uses it) over
liborbhip.so: ``transform`` gives the BowVector / FeatureVector of a frame's descriptors
(U:src/Frame.cc::ComputeBoW, levelsup 4) from the GPU per-descriptor transform."""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import Context, check, lib, ptr
from .vocabulary import Vocabulary, bow_vector, feature_vector


class ORBVocabulary:
    def __init__(self, vocab: Vocabulary | str, device: int = -1, ctx: Context | None = None):
        self.ctx = ctx or Context(device)
        self._h = ctypes.c_void_p()
        if isinstance(vocab, str):
            check(lib().orbhip_vocab_load_text(self.ctx.handle, vocab.encode(), ctypes.byref(self._h)),
                  "orbhip_vocab_load_text")
        else:
            v = vocab
            par = np.ascontiguousarray(v.parent, np.int32)
            leaf = np.ascontiguousarray(v.is_leaf, np.uint8)
            desc = np.ascontiguousarray(v.desc, np.uint8)
            w = np.ascontiguousarray(v.weight, np.float64)
            check(lib().orbhip_vocab_create(self.ctx.handle, v.k, v.L, v.scoring, v.weighting, v.n_nodes, ptr(par),
                                            ptr(leaf), ptr(desc), ptr(w), ctypes.byref(self._h)),
                  "orbhip_vocab_create")
        k, L, nn, nw = (ctypes.c_int32() for _ in range(4))
        check(lib().orbhip_vocab_info(self._h, ctypes.byref(k), ctypes.byref(L), ctypes.byref(nn), ctypes.byref(nw)),
              "orbhip_vocab_info")
        self.k, self.L, self.n_nodes, self.n_words = k.value, L.value, nn.value, nw.value

    @property
    def handle(self):
        return self._h

    def size(self) -> int:
        return self.n_words

    def transform_features(self, desc, levelsup: int = 4):
        """Per descriptor: (word id, FeatureVector node, weight)."""
        d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        n = d.shape[0]
        w = np.zeros(n, np.int32); nd = np.zeros(n, np.int32); wt = np.zeros(n, np.float64)
        check(lib().orbhip_bow_transform(self.ctx.handle, self._h, ptr(d), n, int(levelsup), ptr(w), ptr(nd), ptr(wt)),
              "orbhip_bow_transform")
        return w, nd, wt

    def transform(self, desc, levelsup: int = 4):
        """(BowVector (words, values), FeatureVector {node: [feature indices]})."""
        w, nd, wt = self.transform_features(desc, levelsup)
        return bow_vector(w, wt), feature_vector(nd, wt)

    def close(self):
        if self._h:
            lib().orbhip_vocab_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
