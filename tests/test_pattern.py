"""KAT: the committed rBRIEF pattern equals the in-container skimage artefact
(orb_descriptor_positions.txt, md5 010b675bf1aa5c588eb6386cc24ce66d == OpenCV bit_pattern_31_)."""
import hashlib
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _table():
    src = open(os.path.join(ROOT, "include", "orbhip_pattern.h")).read()
    body = src[src.index("ORBHIP_BIT_PATTERN_31_INIT {"):src.index("}\n#ifndef")]
    return [int(v) for v in re.findall(r"-?\d+", body.split("{", 1)[1])]


def test_pattern_md5_matches_artefact():
    vals = _table()
    assert len(vals) == 1024
    text = "".join(" ".join("%.18e" % float(v) for v in vals[4 * i: 4 * i + 4]) + "\n" for i in range(256))
    assert hashlib.md5(text.encode()).hexdigest() == "010b675bf1aa5c588eb6386cc24ce66d"


def test_pattern_first_last_rows_and_radius():
    vals = _table()
    assert vals[:12] == [8, -3, 9, 5, 4, 2, 7, -12, -11, 9, -8, 2]
    assert vals[-4:] == [-1, -6, 0, -11]
    assert min(vals) >= -13 and max(vals) <= 12
    r = max((vals[2 * i] ** 2 + vals[2 * i + 1] ** 2) ** 0.5 for i in range(512))
    assert abs(r - 18.385) < 1e-3   # max rotated offset 18 < EDGE_THRESHOLD 19
