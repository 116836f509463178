"""Streaming history writer (zarr-v2 layout of the reference's lightsheet sweep): round trips."""
import json
import os

import numpy as np
import pytest

from ray_trace_pb_amd.io import ARRAY_COLUMNS, HistoryWriter, read_array, read_attrs
from parity import same_bits  # noqa: E402


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
        assert same_bits(got[i], hist[i])
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
        assert same_bits(got[i], ref[i])


LIGHTSHEET_RADII = (8.0, 120.0, 1e9)
# scripts/2024_04_01_lightsheet.py:23-36 (the script's settings dict, stored as the store's attrs)
LIGHTSHEET_SETTINGS = {"nrays": 1001, "wavelength": 0.532, "aperture_radius_etl": 8, "aperture_radius": 50.8 / 2,
                       "n_etl": 1.3, "t_edge": 5, "f1": 160, "f2": 120, "fobj": 20, "t_coverglass": 1.25,
                       "n_coverglass": 1.4585, "dz_coverglass": 10, "n_immersion": 1.333}


def _lightsheet_golden(r):
    from parity import GOLDEN
    d = np.load(os.path.join(GOLDEN, "lightsheet_r%s.npz" % {8.0: "8", 120.0: "120", 1e9: "1e9"}[r]))
    return d["rays_in"], d["history"], str(d["system_json"])


def _check_lightsheet_store(p, histories):
    meta = json.load(open(os.path.join(p, "rays", ".zarray")))
    # the script's z.create("rays", shape=(n_config, 17, nrays, 8), chunks=(1, 17, nrays, 8), dtype=float)
    assert meta["shape"] == [3, 17, 1001, 8] and meta["chunks"] == [1, 17, 1001, 8] and meta["dtype"] == "<f8"
    assert read_attrs(p, "rays")["array_columns"] == ["x", "y", "z", "dx", "dy", "dz", "phase", "wavelength"]
    assert read_attrs(p)["settings"] == LIGHTSHEET_SETTINGS
    rc = read_array(p, "radius_curvatures")
    assert np.array_equal(rc, np.array(LIGHTSHEET_RADII))
    assert np.array_equal(read_array(p, "focal_lens_mm"), rc / (LIGHTSHEET_SETTINGS["n_etl"] - 1))
    got = read_array(p)
    for i, h in enumerate(histories):
        assert same_bits(got[i], h), i


def _write_lightsheet_store(p, histories):
    rc = np.array(LIGHTSHEET_RADII)
    focal = rc / (LIGHTSHEET_SETTINGS["n_etl"] - 1)
    with HistoryWriter(p, len(rc), 17, 1001, attrs={"settings": LIGHTSHEET_SETTINGS}) as w:
        w.write_array("radius_curvatures", rc)
        w.write_array("etl_diopters", 1e3 / focal)
        w.write_array("focal_lens_mm", focal)
        for i, h in enumerate(histories):
            w.write(i, h)


def test_lightsheet_store_layout_from_reference_histories(tmp_path):
    """The reference's own lightsheet histories (golden vectors of the script's system at three ETL radii)
    stored in the script's layout and read back bit for bit."""
    hist = [_lightsheet_golden(r)[1] for r in LIGHTSHEET_RADII]
    _write_lightsheet_store(tmp_path / "ref.zarr", hist)
    _check_lightsheet_store(tmp_path / "ref.zarr", hist)


@pytest.mark.gpu
def test_lightsheet_sweep_traced_on_gpu_and_streamed_matches_reference(tmp_path):
    """scripts/2024_04_01_lightsheet.py:51-60,134-135 on the GPU: the three golden ETL systems, rebuilt with
    the drop-in API, traced as device histories and streamed through HistoryWriter (pinned async D2H +
    writer thread) into one 3-configuration store; the read-back equals the REFERENCE's histories."""
    torch = pytest.importorskip("torch")
    import ray_trace_pb_amd.materials as mat
    import ray_trace_pb_amd.raytrace as rt
    import systems
    from serialize import system_to_json
    dev_hist, ref_hist = [], []
    for r in LIGHTSHEET_RADII:
        rays, ref, sys_json = _lightsheet_golden(r)
        system, rays_rec, m0, m1 = systems.lightsheet(rt, mat, r)
        assert json.loads(system_to_json(system, m0, m1)) == json.loads(sys_json)
        assert np.array_equal(rays_rec, rays)
        dev_hist.append(system.ray_trace(torch.from_numpy(rays).cuda(), m0, m1))
        ref_hist.append(ref)
    _write_lightsheet_store(tmp_path / "gpu.zarr", dev_hist)
    _check_lightsheet_store(tmp_path / "gpu.zarr", ref_hist)


def test_zlib_chunks_split_along_rays(tmp_path):
    """compressor="zlib": zarr's numcodecs.Zlib chunk encoding (one zlib stream per chunk, {"id": "zlib", "level"});
    chunk_rays splits a configuration along the ray axis, the last chunk padded to full size with the fill value as
    zarr stores edge chunks.  (zarr / numcodecs are not installed: the codec's parity is pinned by these round trips
    and by zlib itself.)"""
    import zlib
    rng = np.random.default_rng(1)
    hist = [rng.normal(size=(5, 23, 8)) for _ in range(3)]
    hist[1][2, 7] = np.nan
    p = tmp_path / "z.zarr"
    with HistoryWriter(p, 4, 5, 23, compressor=("zlib", 6), chunk_rays=10, workers=3) as w:
        for i in range(3):
            w.write(i, hist[i])
    meta = json.load(open(os.path.join(p, "rays", ".zarray")))
    assert meta["compressor"] == {"id": "zlib", "level": 6} and meta["chunks"] == [1, 5, 10, 8]
    assert sorted(f for f in os.listdir(os.path.join(p, "rays")) if not f.startswith(".")) == \
        [f"{i}.0.{j}.0" for i in range(3) for j in range(3)]
    # the last chunk of configuration 1: rays 20..22, then NaN padding
    raw = zlib.decompress(open(os.path.join(p, "rays", "1.0.2.0"), "rb").read())
    block = np.frombuffer(raw, dtype="<f8").reshape(5, 10, 8)
    assert same_bits(block[:, :3], hist[1][:, 20:]) and np.isnan(block[:, 3:]).all()
    got = read_array(p)
    for i in range(3):
        assert same_bits(got[i], hist[i])
    assert np.isnan(got[3]).all()


def test_compressor_argument_checks(tmp_path):
    with pytest.raises(ValueError):
        HistoryWriter(tmp_path / "a.zarr", 1, 1, 1, compressor="blosc")
    with pytest.raises(ValueError):
        HistoryWriter(tmp_path / "b.zarr", 1, 1, 1, compressor=("zlib", 12))
    w = HistoryWriter(tmp_path / "c.zarr", 1, 3, 4, compressor={"id": "zlib", "level": 1})
    w.write(0, np.ones((3, 4, 8)))
    w.close()
    assert same_bits(read_array(tmp_path / "c.zarr")[0], np.ones((3, 4, 8)))


@pytest.mark.gpu
def test_device_histories_to_zlib_chunks(tmp_path):
    """Device histories through the pinned D2H path into zlib chunks split along the rays."""
    torch = pytest.importorskip("torch")
    import ray_trace_pb_amd.materials as mat
    import ray_trace_pb_amd.raytrace as rt
    import systems
    system, rays, m0, m1 = systems.c1_plano_convex(rt, mat)
    x = torch.from_numpy(rays).cuda()
    ref = []
    p = tmp_path / "gpu_z.zarr"
    with HistoryWriter(p, 2, 7, rays.shape[0], compressor="zlib", chunk_rays=300, workers=4) as w:
        for i in range(2):
            h = system.ray_trace(x + torch.tensor([0, 0, -i, 0, 0, 0, 0, 0], dtype=x.dtype, device=x.device), m0, m1)
            ref.append(h.cpu().numpy())
            w.write(i, h)
    got = read_array(p)
    for i in range(2):
        assert same_bits(got[i], ref[i])
