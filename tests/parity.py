"""Shared parity helpers (the comparison rule of SURVEY.md §8c)."""
import glob
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
ALL_CASES = sorted(os.path.basename(f)[:-4] for f in glob.glob(os.path.join(GOLDEN, "*.npz"))
                   if os.path.basename(f)[:-4] not in ("shapes", "generators"))
# float64-input recipes (the reference run on float64 rays) and their float32-input variants (the same
# recipe's rays rounded to float32 and handed to the reference as float32 arrays)
CASES = [c for c in ALL_CASES if not c.endswith("_f32in")]
F32IN_CASES = [c for c in ALL_CASES if c.endswith("_f32in")]


def load_case(name):
    d = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    spec = json.loads(str(d["system_json"]))
    return spec, d["rays_in"], d["history"]


def same_bits(got, ref):
    """Bit-identical: equal shapes, NaN exactly where ref has NaN, and every other element the same bit
    pattern (so +0 and -0 differ; np.array_equal with equal_nan=True treats them as equal).  Float arrays
    of different widths are compared after an exact widening to the wider type."""
    got, ref = np.asarray(got), np.asarray(ref)
    if got.shape != ref.shape:
        return False
    if not (np.issubdtype(got.dtype, np.floating) and np.issubdtype(ref.dtype, np.floating)):
        return bool(np.array_equal(got, ref))
    t = np.result_type(got.dtype, ref.dtype)
    got, ref = got.astype(t, copy=False), ref.astype(t, copy=False)
    nan = np.isnan(ref)
    if not np.array_equal(np.isnan(got), nan):
        return False
    u = {2: np.uint16, 4: np.uint32, 8: np.uint64}[t.itemsize]
    return bool(np.array_equal(np.ascontiguousarray(got[~nan]).view(u), np.ascontiguousarray(ref[~nan]).view(u)))


def compare(got, ref, rtol):
    """NaN masks must be equal element for element; finite values must satisfy
    |got - ref| <= rtol * max(|ref|, colmax) where colmax is the max |finite ref| of that column in
    that plane (column-scaled tolerance).  Returns (ok, report dict)."""
    got = np.asarray(got, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    if got.shape != ref.shape:
        return False, {"shape": (got.shape, ref.shape)}
    nan_g, nan_r = np.isnan(got), np.isnan(ref)
    mask_flips = int((nan_g != nan_r).sum())
    fin = ~nan_g & ~nan_r
    absref = np.where(np.isfinite(ref), np.abs(ref), 0.0)
    colmax = absref.max(axis=-2, keepdims=True) if ref.ndim >= 2 else absref.max()
    scale = np.maximum(absref, colmax)
    with np.errstate(invalid="ignore"):
        err = np.where(fin & (got != ref), np.abs(got - ref), 0.0)      # equal infinities: no error
    inf_mismatch = int((fin & (np.isinf(got) | np.isinf(ref)) & (got != ref)).sum())
    err = np.where(np.isinf(err), 0.0, err)
    with np.errstate(invalid="ignore", divide="ignore"):
        rel = np.where(scale > 0, err / scale, err)
    max_rel = float(rel.max()) if rel.size else 0.0
    n_bit_diff = int((fin & (got != ref)).sum())
    ok = mask_flips == 0 and inf_mismatch == 0 and max_rel <= rtol
    return ok, {"mask_flips": mask_flips, "max_rel": max_rel, "n_values_not_bitwise": n_bit_diff,
                "inf_mismatch": inf_mismatch}
