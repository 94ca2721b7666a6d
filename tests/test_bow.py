"""Bag of words: DBoW2 transform + BowVector / FeatureVector and
ORBmatcher::SearchByBoW. CPU: known-answer tests of the oracle restatement on hand-built
vocabularies, the ORBvoc.txt text round trip. GPU: bit-exact word / node / weight per descriptor
and identical SearchByBoW matches vs the oracle. Parity unpinned by the reference (DBoW2 and
ORBvoc.txt are absent): the vocabularies are synthetic (orb_slam3_ros2_amd.vocabulary)."""
import numpy as np
import pytest

from orb_slam3_ros2_amd.vocabulary import Vocabulary, bow_vector, feature_vector


def _tiny_vocab():
    """k=2, L=2: root -> {1, 2}; 1 -> {3, 4}; 2 -> {5, 6}. Node 2's descriptor equals node 1's
    (ties: the first child wins); leaves 3..6 are words 0..3 (leaf order); node 6 has weight 0."""
    desc = np.zeros((7, 32), np.uint8)
    desc[1] = 0x00; desc[2] = 0x00
    desc[3, :4] = 0x0F; desc[4, :4] = 0xF0
    desc[5] = 0xFF; desc[6] = 0xAA
    parent = np.array([-1, 0, 0, 1, 1, 2, 2], np.int32)
    leaf = np.array([0, 0, 0, 1, 1, 1, 1], np.uint8)
    weight = np.array([0, 0, 0, 1.5, 2.0, 3.0, 0.0])
    return Vocabulary(2, 2, 0, 0, parent, leaf, desc, weight)


def test_oracle_transform_known_answers(oracle):
    v = _tiny_vocab()
    f = np.zeros((3, 32), np.uint8)
    f[0, :4] = 0x0F              # -> node 1 (tie with 2, first wins) -> leaf 3 (word 0)
    f[1, :4] = 0xF0              # -> node 1 -> leaf 4 (word 1)
    f[2] = 0xAA                  # node 1 and 2 tie (both 0x00) -> 1 -> 3 vs 4 tie -> 3
    w, nd, wt = oracle.bow_transform(v, f, levelsup=1)   # FeatureVector level L - 1 = 1
    assert w.tolist() == [0, 1, 0] and nd.tolist() == [1, 1, 1]
    assert wt.tolist() == [1.5, 2.0, 1.5]
    w2, nd2, _ = oracle.bow_transform(v, f, levelsup=4)  # level <= 0 -> root
    assert nd2.tolist() == [0, 0, 0]
    words, vals = oracle.bow_vector(w, wt)
    assert words.tolist() == [0, 1] and np.allclose(vals, [3.0 / 5.0, 2.0 / 5.0])
    ww, vv = bow_vector(w, wt)
    assert ww.tolist() == words.tolist() and np.allclose(vv, vals)
    assert feature_vector(nd, wt) == {1: [0, 1, 2]}


def test_zero_weight_words_leave_both_vectors(oracle):
    v = _tiny_vocab()
    v.desc[1] = 0xFF             # node 1 = 0xFF, node 2 = 0x00
    f = np.zeros((2, 32), np.uint8)
    f[0, :] = 0xAA               # d = 128 to both -> node 1 (first) -> a weighted leaf
    f[1] = 0x00                  # node 2 -> leaf 6 (0xAA, d 128 < 256): weight 0, in neither vector
    w, nd, wt = oracle.bow_transform(v, f, levelsup=1)
    keep = wt > 0
    words, _ = oracle.bow_vector(w, wt)
    assert set(words.tolist()) == set(w[keep].tolist())
    assert sum(len(x) for x in feature_vector(nd, wt).values()) == int(keep.sum())


def test_vocabulary_text_round_trip(tmp_path):
    v = Vocabulary.synthetic(k=4, L=3, seed=2)
    p = str(tmp_path / "voc.txt")
    v.save_text(p)
    u = Vocabulary.load_text(p)
    assert (u.k, u.L) == (4, 3) and np.array_equal(u.parent, v.parent) and np.array_equal(u.desc, v.desc)
    assert np.array_equal(u.is_leaf, v.is_leaf) and np.allclose(u.weight, v.weight, rtol=0, atol=0)
    first, nch, children, word = v.csr()
    assert nch[0] == 4 and word.max() == 4 ** 3 - 1


def test_oracle_search_bow_greedy_and_ratio(oracle):
    """Two KF features in one node compete for the same frame feature: the first (index order)
    takes it, the second falls back to the remaining one; ratio rejects an ambiguous pair."""
    kd = np.zeros((3, 32), np.uint8)
    kd[1] = kd[0]; kd[1, 0] ^= 0x01            # near-duplicate of KF 0
    kd[2] = 0x55
    fd = np.zeros((3, 32), np.uint8)
    fd[1] = fd[0]; fd[1, 0] ^= 0x03            # 2 bits from frame 0
    fd[2] = 0x55; fd[2, 0] ^= 0x01
    ka = np.zeros(3, np.float32); fa = np.zeros(3, np.float32)
    n, m = oracle.search_bow(kd, ka, np.array([5, 5, 9]), np.array([1, 1, 1], np.uint8), fd, fa,
                             np.array([5, 5, 9]), ratio=0.9, check_orientation=False)
    # KF0 -> frame 0 (d 0 vs 2: accepted); KF1 -> frame 1 (frame 0 taken; d=1, second 256);
    # KF2 -> frame 2 (only candidate, d = 1)
    assert m.tolist() == [0, 1, 2] and n == 3
    n2, m2 = oracle.search_bow(kd, ka, np.array([5, 5, 9]), np.array([0, 1, 1], np.uint8), fd, fa,
                               np.array([5, 5, 9]), ratio=0.6, check_orientation=False)
    # KF0 has no map point; KF1: d(f0)=1, d(f1)=1 -> best 1, second 1: 1 < 0.6 fails
    assert m2.tolist() == [-1, -1, 2] and n2 == 1


# ------------------------------------------------------------------------------- GPU
def _frames():
    from orb_slam3_ros2_amd import ORBextractor
    from orb_slam3_ros2_amd.synthetic import shifted_frame, synthetic_frame
    ext = ORBextractor(1000)
    a = synthetic_frame(41)
    b = shifted_frame(a, 3, 2, 42)
    _, ka, da = ext(a)
    _, kb, db = ext(b)
    return ka, da, kb, db


@pytest.mark.gpu
@pytest.mark.parametrize("k,L,levelsup", [(10, 6, 4), (10, 4, 2), (6, 5, 3)])
def test_gpu_transform_bit_exact(oracle, k, L, levelsup):
    from orb_slam3_ros2_amd import ORBVocabulary
    v = Vocabulary.synthetic(k, L, seed=7)
    ka, da, kb, db = _frames()
    rng = np.random.default_rng(3)
    feats = np.concatenate([da, db, rng.integers(0, 256, (500, 32), dtype=np.uint8)])
    voc = ORBVocabulary(v)
    w, nd, wt = voc.transform_features(feats, levelsup)
    ow, on, ov = oracle.bow_transform(v, feats, levelsup)
    assert np.array_equal(w, ow) and np.array_equal(nd, on) and np.array_equal(wt, ov)
    (gw, gv), gfv = voc.transform(feats, levelsup)
    rw, rv = oracle.bow_vector(ow, ov)
    assert np.array_equal(gw, rw) and np.array_equal(gv, rv)


@pytest.mark.gpu
def test_gpu_vocab_load_text(tmp_path, oracle):
    from orb_slam3_ros2_amd import ORBVocabulary
    v = Vocabulary.synthetic(8, 4, seed=9)
    p = str(tmp_path / "voc.txt")
    v.save_text(p)
    voc = ORBVocabulary(p)
    assert (voc.k, voc.L, voc.n_nodes, voc.n_words) == (8, 4, v.n_nodes, 8 ** 4)
    rng = np.random.default_rng(5)
    f = rng.integers(0, 256, (300, 32), dtype=np.uint8)
    w, nd, wt = voc.transform_features(f, 2)
    ow, on, ov = oracle.bow_transform(v, f, 2)
    assert np.array_equal(w, ow) and np.array_equal(nd, on) and np.array_equal(wt, ov)


@pytest.mark.gpu
@pytest.mark.parametrize("ratio,ori,levelsup", [(0.7, True, 4), (0.9, False, 4), (0.75, True, 3)])
def test_gpu_search_bow_matches_oracle(oracle, ratio, ori, levelsup):
    from orb_slam3_ros2_amd import ORBmatcher, ORBVocabulary
    v = Vocabulary.synthetic(10, 6, seed=11)
    voc = ORBVocabulary(v)
    ka, da, kb, db = _frames()
    kw_, kn, kwt = voc.transform_features(da, levelsup)
    fw_, fn, fwt = voc.transform_features(db, levelsup)
    valid = (np.random.default_rng(6).random(len(da)) < 0.8).astype(np.uint8)
    mt = ORBmatcher(ratio, ori, ctx=voc.ctx)
    n, m = mt.SearchByBoW(da, ka["angle"], kn, kwt, valid, db, kb["angle"], fn, fwt)
    # the oracle takes FeatureVector membership from node >= 0: gate by weight on both sides
    on2, om2 = oracle.search_bow(da, ka["angle"], np.where(kwt > 0, kn, -1), valid, db, kb["angle"],
                                 np.where(fwt > 0, fn, -1), ratio=ratio, check_orientation=ori)
    assert n == on2 and np.array_equal(m, om2)
    assert n > 50
