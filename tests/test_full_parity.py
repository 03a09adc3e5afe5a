"""The full-set LM parity tables of DESIGN.md §4 (tools/full_parity.py over every DLT inlier of the
C4 frame pair: DETMATH, the GPU contract, against STRICT, libm's transcendentals, and against the
opt-in tree-reduction mode DETMATH|TREE|GRAM), pinned two ways.  CPU only (the oracle):

  * the per-point arrays the tool saved (tests/golden/full_parity_c4.npz) reproduce every count of
    the committed table (profiles/r05_full_parity.json), so the figures DESIGN.md quotes are the
    data's;
  * a pinned subset -- the 16 largest STRICT moves, the 16 largest tree moves and 32 seeded points --
    re-run through the oracle in all three modes gives the saved statuses and normals bit for bit.
"""
import json
import os

import numpy as np
import pytest

from conftest import oracle_threads

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIXTURE = os.path.join(ROOT, "tests", "golden", "full_parity_c4.npz")
TABLE = os.path.join(ROOT, "profiles", "r05_full_parity.json")
TREE, GRAM = 64, 128  # oracle/fm3d_oracle.c ORC_LM_TREE / ORC_LM_GRAM

pytestmark = pytest.mark.skipif(not (os.path.exists(FIXTURE) and os.path.exists(TABLE)),
                                reason="tools/full_parity.py has not been run")


class Cam:
    def __init__(self, arr):
        self.fx, self.fy, self.cx, self.cy = arr[:4]
        self.k = tuple(arr[4:9])


@pytest.fixture(scope="module")
def fx():
    return np.load(FIXTURE, allow_pickle=False)


@pytest.fixture(scope="module")
def table():
    with open(TABLE) as f:
        return json.load(f)


def _counts(sb, so, d):
    both = (sb == 0) & (so == 0)
    dk = d[both]
    return {
        "points": len(sb),
        "status_equal": int((sb == so).sum()),
        "keep_drop_changed": int(((sb == 0) != (so == 0)).sum()),
        "kept_both": int(both.sum()),
        "normals_bit_equal": int((dk == 0).sum()),
        "within_1e-4": int((dk <= 1e-4).sum()),
        "beyond_1e-4": int((dk > 1e-4).sum()),
        "max": float(dk.max()),
    }


@pytest.mark.parametrize("other,key", [("strict", "strict_vs_detmath"), ("tree", "tree_gram_vs_detmath")])
def test_table_is_the_saved_data(fx, table, other, key):
    c = _counts(fx["status_detmath"], fx[f"status_{other}"], fx[f"dn_{other}"])
    for k, v in c.items():
        assert table[key][k] == v, (key, k)
    assert table["inliers"] == len(fx["status_detmath"]) == 71223


def test_strict_vs_detmath_bar(table):
    """The GPU contract (DETMATH: correctly rounded sin / cos / atan2 / exp, include/fm3d_crmath.h)
    against libm on all 71,223 C4 inliers (DESIGN.md §4 quotes the table): the same status on every
    point, every kept normal within 1e-4 -- in fact within 1e-15, 35,808 of 36,151 bit for bit.  The
    345 points that differ at all differ through libm's sin, cos and atan2 (not correctly rounded
    on every argument here), not exp (the attribution runs)."""
    t = table["strict_vs_detmath"]
    assert t["status_changed"] == 0 and t["keep_drop_changed"] == 0
    assert t["beyond_1e-4"] == 0 and t["frac_within_1e-4"] == 1.0 and t["max"] < 1e-15
    a = table["attribution"]
    assert a["points_differing_at_all"] == 345 and a["large_points"] == 0
    assert a["sample:exp"]["vs_strict"]["normals_bit_equal"] == 0  # libm's exp alone explains none
    assert a["sample:sin+cos"]["vs_strict"]["normals_bit_equal"] > a["sample:sin"]["vs_strict"]["normals_bit_equal"]


def test_tree_mode_gate_fails(table):
    """VERDICT r04 item 1's gate for the tree-reduction mode (DETMATH | TREE | GRAM against the
    default order, all 71,223 inliers): it asks for identical statuses and every kept normal within
    1e-4.  22 points change keep/drop and 7,507 of the 36,140 kept by both move past 1e-4 (median
    3e-14), so the mode stays opt-in."""
    t = table["tree_gram_vs_detmath"]
    assert t["keep_drop_changed"] == 22 and t["beyond_1e-4"] == 7507 and t["kept_both"] == 36140


def test_pinned_subset_reruns_bitwise(orc, fx):
    cam = Cam(fx["cam"])
    P = fx["pin_points"]
    for mode, tag in ((orc.DETMATH, "detmath"), (orc.STRICT, "strict"), (orc.DETMATH | TREE | GRAM, "tree")):
        r = orc.optimize_normals(cam, fx["R2"], fx["t2"], fx["img1"], fx["img2"], 3, P, 64, mode=mode,
                                 nthreads=oracle_threads())
        assert np.array_equal(r["status"], fx[f"pin_status_{tag}"]), tag
        ok = r["status"] == 0
        assert np.array_equal(r["normals"][ok], fx[f"pin_normals_{tag}"][ok]), tag
