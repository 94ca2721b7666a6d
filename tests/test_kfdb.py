"""KeyFrameDatabase place recognition: U:src/KeyFrameDatabase.cc
DetectRelocalizationCandidates and DetectNBestCandidates with DBoW2 L1 scoring.

CPU: the oracle against definitional checks (a query equal to a KeyFrame's BowVector scores 1
against it and retrieves it; an empty database returns nothing; erased KeyFrames never come
back). GPU: a sequence of queries (so the persistent KeyFrame members, including the stale
scores upstream keeps for shared-but-unscored KeyFrames, carry over) with adds and erases in
between, device vs oracle, identical candidate lists. Parity unpinned by the reference (no
fixtures upstream).
"""
import numpy as np
import pytest

from orb_slam3_ros2_amd.synthetic import synthetic_kfdb_scene, synthetic_query_bow


def _l1(a, b):
    wa, va = a
    wb, vb = b
    common, ia, ib = np.intersect1d(wa, wb, return_indices=True)
    s = 0.0
    for x, y in zip(va[ia], vb[ib]):
        s += abs(x - y) - abs(x) - abs(y)
    return -s / 2.0


def test_oracle_relocalization_definitional(oracle):
    sc = synthetic_kfdb_scene(n_kf=60, seed=1)
    db = oracle.KeyFrameDatabase(60, 20000)
    assert len(db.DetectRelocalizationCandidates(1, sc["bows"][5], sc["covis"])) == 0   # empty
    for i, b in enumerate(sc["bows"]):
        db.add(i, b)
    assert abs(_l1(sc["bows"][30], sc["bows"][30]) - 1.0) < 1e-12
    c = db.DetectRelocalizationCandidates(2, sc["bows"][30], sc["covis"])
    assert len(c) > 0 and (np.abs(c - 30) <= 10).all()
    db.erase(30)
    for j in sc["covis"][30]:
        db.erase(int(j))
    c = db.DetectRelocalizationCandidates(3, sc["bows"][30], sc["covis"])
    assert 30 not in c.tolist()


def test_oracle_nbest_excludes_connected(oracle):
    sc = synthetic_kfdb_scene(n_kf=80, seed=2)
    db = oracle.KeyFrameDatabase(80, 20000)
    for i, b in enumerate(sc["bows"][:70]):
        db.add(i, b)
    q = 75
    con = np.zeros(80, np.uint8)
    con[sc["covis"][q][sc["covis"][q] >= 0]] = 1
    lo, me = db.DetectNBestCandidates(1000 + q, sc["bows"][q], sc["covis"], con, 3, sc["kf_map"], int(sc["kf_map"][q]))
    assert len(lo) <= 3 and len(me) <= 3
    assert not con[lo].any() and not con[me].any()
    assert (sc["kf_map"][lo] == sc["kf_map"][q]).all() and (sc["kf_map"][me] != sc["kf_map"][q]).all()


@pytest.mark.gpu
def test_kfdb_matches_oracle(oracle):
    from orb_slam3_ros2_amd import KeyFrameDatabase
    n_kf = 240
    sc = synthetic_kfdb_scene(n_kf=n_kf, seed=5)
    dev = KeyFrameDatabase(n_kf)
    ref = oracle.KeyFrameDatabase(n_kf, 20000)
    rng = np.random.Generator(np.random.PCG64(9))
    qid = 10
    added = []
    sizes = []
    for i in range(n_kf):
        dev.add(i, sc["bows"][i]); ref.add(i, sc["bows"][i]); added.append(i)
        if i % 40 == 39:
            # a burst of relocalisation queries and loop queries on the database so far
            for t in range(6):
                ks = rng.choice(i + 1, 1 + t % 3, replace=False)   # one place, or several
                k = int(ks[0])
                bow = synthetic_query_bow(sc, ks, seed=qid, keep=0.5)
                km = sc["kf_map"] if t % 2 else None
                a = dev.DetectRelocalizationCandidates(qid, bow, sc["covis"], km, int(sc["kf_map"][k]))
                b = ref.DetectRelocalizationCandidates(qid, bow, sc["covis"], km, int(sc["kf_map"][k]))
                assert np.array_equal(a, b), (i, t, a, b)
                sizes.append(len(a))
                qid += 1
                con = np.zeros(n_kf, np.uint8)
                con[sc["covis"][k][sc["covis"][k] >= 0]] = 1
                flags = (rng.random(n_kf) < 0.05).astype(np.uint8)
                a = dev.DetectNBestCandidates(qid, bow, sc["covis"], con, 3, sc["kf_map"], int(sc["kf_map"][k]), flags)
                b = ref.DetectNBestCandidates(qid, bow, sc["covis"], con, 3, sc["kf_map"], int(sc["kf_map"][k]), flags)
                assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]), (i, t, a, b)
                sizes.append(len(a[0]) + len(a[1]))
                qid += 1
            # KeyFrame culling
            for k in rng.choice(added, 3, replace=False):
                dev.erase(int(k)); ref.erase(int(k)); added.remove(int(k))
    assert max(sizes) >= 3 and np.mean(sizes) > 1.2   # lists with several candidates were compared
