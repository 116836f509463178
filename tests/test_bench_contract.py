"""bench.py contract on the CPU: the roofline object's fields and the algorithmic-byte accounting of the
headline workload.  The timed run itself needs a GPU (driver / gpurun)."""
import types

import bench


def test_c3_workload_size_and_bytes():
    nt, nph = bench.C3_FAN
    rays = 5 * nt * nph                                  # 5 field points x get_ray_fan(h, 1 deg, 3163, nphis=3162)
    assert rays == 50_007_030
    S, planes = 9, 19
    per_ray = 8 * 8 + planes * 8 * 4                     # float64 input record + 19 float32 history records
    assert per_ray == 672
    assert rays * per_ray == 33_604_724_160              # alg_bytes_per_launch in profiles/r02/bench.log
    assert abs(per_ray / S - 74.667) < 1e-3


def test_roofline_object_fields():
    wl = types.SimpleNamespace(alg_bytes=33_604_724_160, bytes_per_ray=672, S=9)
    r = bench.roofline(wl, 6.2, traffic=3.36e10, traffic_note=None, fill=6800.0, copy=4700.0)
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == bench.HBM_PEAK_GBS
    assert abs(r["achieved"] - 33_604_724_160 / 6.2e-3 / 1e9) < 1e-6
    assert abs(r["frac"] - r["achieved"] / 8000.0) < 1e-12
    assert abs(r["frac_of_output_fill"] - r["achieved"] / 6800.0) < 1e-12
    assert abs(r["frac_of_torch_copy"] - r["achieved"] / 4700.0) < 1e-12
    assert "torch_copy_GBps" not in bench.roofline(wl, 6.2)
