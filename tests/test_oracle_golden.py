"""The NumPy oracle reproduces the reference's own outputs (golden vectors) BIT FOR BIT."""
import numpy as np
import pytest

from oracle import rt_numpy as O
from parity import same_bits, CASES, F32IN_CASES, compare, load_case


@pytest.mark.parametrize("name", CASES)
def test_oracle_matches_reference_bitwise(name):
    spec, rays, ref = load_case(name)
    got = O.ray_trace(spec["surfaces"], spec["materials"], rays)
    assert got.shape == ref.shape
    assert same_bits(got, ref)


@pytest.mark.parametrize("name", F32IN_CASES)
def test_oracle_on_widened_float32_input_vs_reference(name):
    """The reference given float32 rays returns a float64 history.  NumPy's promotion rules make it
    evaluate a few first-surface sub-expressions in float32 (``2 * np.pi / wls`` in PerfectLens RT:1773,
    ``wavelength ** 2`` in Sellmeier MAT:48-50); every later surface sees the float64 history.  The
    oracle (and the GPU) widen the float32 input exactly and compute everything in float64: NaN masks
    must be identical and values within 1e-6 column-scaled (float32 bar: 1e-5)."""
    spec, rays, ref = load_case(name)
    assert rays.dtype == np.float32 and ref.dtype == np.float64
    got = O.ray_trace(spec["surfaces"], spec["materials"], rays.astype(np.float64))
    ok, rep = compare(got, ref, rtol=1e-6)
    assert ok and rep["mask_flips"] == 0, rep


def test_oracle_input_ranks():
    import json, os
    from parity import GOLDEN
    d = np.load(os.path.join(GOLDEN, "shapes.npz"))
    spec = json.loads(str(d["system_json"]))
    for k in ("1", "2", "3"):
        got = O.ray_trace(spec["surfaces"], spec["materials"], d["rays" + k])
        assert same_bits(got, d["out" + k]), k


def test_oracle_generators():
    import os
    from parity import GOLDEN
    d = np.load(os.path.join(GOLDEN, "generators.npz"))
    assert np.array_equal(O.ray_fan([1., 2., 3.], 0.3, 7, 0.5, nphis=5), d["fan"])


def test_golden_cases_exercise_edge_semantics():
    """The fixtures must contain the per-ray failure modes the kernel has to reproduce."""
    _, _, h = load_case("tir_prism")
    # TIR: refracted plane keeps phase and wavelength but position is NaN (RT:1221)
    tir = np.isnan(h[4, :, 0]) & ~np.isnan(h[4, :, 6]) & ~np.isnan(h[4, :, 7])
    assert tir.sum() > 0
    _, _, h = load_case("stress")
    miss = np.isnan(h[:, :, 0]) & ~np.isnan(h[:, :, 3])      # sphere miss keeps d and wavelength
    assert miss.sum() > 0
    _, _, h = load_case("c4_opm")
    assert np.isnan(h[-1]).all(axis=1).sum() > 0              # NA clip of PerfectLens (RT:1757-1760)
