"""Streaming history writer (zarr-v2 layout of the reference's lightsheet sweep): round trips."""
import json
import os

import numpy as np
import pytest

from ray_trace_pb_amd.io import ARRAY_COLUMNS, HistoryWriter, read_array, read_attrs


def test_round_trip_numpy(tmp_path):
    rng = np.random.default_rng(0)
    hist = [rng.normal(size=(7, 13, 8)) for _ in range(4)]
    hist[2][3, 5] = np.nan
    p = tmp_path / "rays.zarr"
    with HistoryWriter(p, 5, 7, 13, attrs={"settings": {"nrays": 13}}) as w:
        for i in (0, 1, 2, 3):
            w.write(i, hist[i])
        w.write_array("radius_curvatures", np.linspace(8, 55, 5))
    got = read_array(p)
    assert got.shape == (5, 7, 13, 8)
    for i in range(4):
        assert np.array_equal(got[i], hist[i], equal_nan=True)
    assert np.isnan(got[4]).all()                                    # unwritten config -> fill value
    assert read_attrs(p, "rays")["array_columns"] == ARRAY_COLUMNS
    assert read_attrs(p)["settings"]["nrays"] == 13
    meta = json.load(open(os.path.join(p, "rays", ".zarray")))
    assert meta["chunks"] == [1, 7, 13, 8] and meta["compressor"] is None and meta["dtype"] == "<f8"
    assert np.array_equal(read_array(p, "radius_curvatures"), np.linspace(8, 55, 5))


def test_shape_checks(tmp_path):
    w = HistoryWriter(tmp_path / "x.zarr", 2, 3, 4)
    with pytest.raises(ValueError):
        w.write(0, np.zeros((3, 5, 8)))
    with pytest.raises(IndexError):
        w.write(2, np.zeros((3, 4, 8)))
    w.close()


@pytest.mark.gpu
def test_round_trip_device_histories(tmp_path):
    torch = pytest.importorskip("torch")
    import sys
    import ray_trace_pb_amd.materials as mat
    import ray_trace_pb_amd.raytrace as rt
    import systems
    system, rays, m0, m1 = systems.c1_plano_convex(rt, mat)
    x = torch.from_numpy(rays).cuda()
    ref = []
    p = tmp_path / "gpu.zarr"
    with HistoryWriter(p, 3, 7, rays.shape[0]) as w:
        for i in range(3):
            h = system.ray_trace(x + torch.tensor([0, 0, -i, 0, 0, 0, 0, 0], dtype=x.dtype, device=x.device), m0, m1)
            ref.append(h.cpu().numpy())
            w.write(i, h)
    got = read_array(p)
    for i in range(3):
        assert np.array_equal(got[i], ref[i], equal_nan=True)
