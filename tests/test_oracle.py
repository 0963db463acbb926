"""Pin the oracle (oracle/rt_oracle.c) against the compiled reference's goldens.

The goldens in tests/golden/ were produced by the unmodified reference
(oracle/_ref/ref_harness, see tests/golden/make_goldens.py).  The oracle must
reproduce them bit-exactly, and its ray counts must equal the counts SURVEY.md
§6 measured with an instrumented copy of the reference.
"""
from __future__ import annotations

import numpy as np
import pytest

from conftest import GOLDEN_DIR, config_path, golden_by_name, load_golden_image

# (golden, camera) -> (primary, shadow, reflection) measured on the instrumented
# reference, SURVEY.md §6 table / BASELINE.md §2.
SURVEY_COUNTS = {
    "C1_simple_aa1": (640_000, 55_185, 0),
    "C2_cornellbox_800_d0_aa1": (640_000, 639_978, 0),
    "hm_verbatim_aa1": (1_036_800, 1_736_616, 796_110),
    "hm_verbatim_aa2": (4_147_200, 6_947_192, 3_184_517),
    "C3_hm_1080p_d6_aa1": (2_073_600, 3_401_420, 1_614_941),
    "C3_hm_1080p_d6_aa2": (8_294_400, 13_605_694, 6_459_686),
    "C5_hm_8k_d6_aa4": (530_841_600, 870_771_386, 413_424_592),
}

CPU_GOLDENS = [
    "C1_simple_aa1", "C1_simple_aa2", "C1_simple_aa3", "C1_simple_aa4", "simple_shading_aa1",
    "simple_reflectance_aa1", "cornellbox_aa1", "C2_cornellbox_800_d0_aa1", "C2_cornellbox_800_d0_aa2",
    "mirror_spheres_aa1", "marbles_aa1", "monkey_aa1", "bunny_aa1", "berserker_aa1", "car_aa1",
    "low_poly_aa1", "dragon_lowres_aa1", "hm_verbatim_aa1", "hm_verbatim_aa2", "C3_hm_1080p_d6_aa1",
    "C3_hm_1080p_d6_aa2",
]


def test_golden_counts_match_survey(goldens):
    for name, (p, s, r) in SURVEY_COUNTS.items():
        c = golden_by_name(goldens, name)["cameras"][0]["counters"]
        assert (c["primary"], c["shadow"], c["reflection"]) == (p, s, r), name


@pytest.mark.parametrize("name", CPU_GOLDENS)
def test_oracle_matches_reference(name, goldens, oracle, scene_dir):
    g = golden_by_name(goldens, name)
    sc = oracle.OracleScene(config_path(scene_dir, g["config"]))
    for cam in g["cameras"]:
        img, counts = sc.render(cam["camera"], aa=g["aa"])
        ref = load_golden_image(cam)
        bad = int((img != ref).any(axis=2).sum())
        assert bad == 0, f"{name}/{cam['image']}: {bad} pixels differ from the reference"
        want = cam["counters"]
        got = (counts["primary_rays"], counts["shadow_rays"], counts["reflection_rays"], counts["node_visits"],
               counts["tri_tests"], counts["sphere_tests"])
        assert got == (want["primary"], want["shadow"], want["reflection"], want["node_visits"],
                       want["tri_tests"], want["sphere_tests"])


@pytest.mark.parametrize("name", ["C1_simple_aa1", "C2_cornellbox_800_d0_aa1", "hm_verbatim_aa1",
                                  "C3_hm_1080p_d6_aa1"])
def test_oracle_primary_hits(name, goldens, oracle, scene_dir):
    import hashlib
    g = golden_by_name(goldens, name)
    ph = g["primary_hits"]
    z = np.load(GOLDEN_DIR / ph["file"], allow_pickle=False)
    sc = oracle.OracleScene(config_path(scene_dir, g["config"]))
    t, m = sc.primary_hits(0, aa=g["aa"])
    flat_t, flat_m = t.reshape(-1), m.reshape(-1)
    assert np.array_equal(flat_t[z["idx"]].view(np.uint32), z["t"].view(np.uint32))
    assert np.array_equal(flat_m[z["idx"]], z["material"])
    assert hashlib.sha256(flat_t.tobytes()).hexdigest() == ph["sha256_t"]
    assert hashlib.sha256(flat_m.tobytes()).hexdigest() == ph["sha256_material"]


def test_oracle_row_range_is_subframe(oracle, scene_dir, goldens):
    """Rendering a row range gives exactly those rows of the full frame (bounded CPU samples)."""
    g = golden_by_name(goldens, "hm_verbatim_aa2")
    sc = oracle.OracleScene(config_path(scene_dir, g["config"]))
    part, _ = sc.render(0, aa=2, rows=(300, 340))
    ref = load_golden_image(g["cameras"][0])
    assert np.array_equal(part, ref[300:340])
