"""C-ABI entry points the Python layer does not call (it uses the bit-exact *_tables forms):
rtpb_ray_fan / rtpb_collimated_rays evaluate cos/sin with the device libm -- within 1 ulp of the host's
(include/rtpb.h), so they agree with the reference generators (RT:45-161) to a few ulps with identical
ray order and exactly equal non-trigonometric fields -- and rtpb_shutdown, after which the library
brings its device state back on the next call."""
import ctypes

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import ray_trace_pb_amd.materials as mat  # noqa: E402
import ray_trace_pb_amd.raytrace as rt  # noqa: E402
from ray_trace_pb_amd import _capi as C  # noqa: E402
from ray_trace_pb_amd import _engine as E  # noqa: E402
import systems  # noqa: E402
from parity import same_bits  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _d3(v):
    return (ctypes.c_double * 3)(*[float(x) for x in v])


@pytest.mark.parametrize("dtype", [C.RTPB_F64, C.RTPB_F32])
def test_device_trig_ray_fan_close_to_reference_generator(dtype):
    pt, th, nt, nph, wl = [0.5, -0.25, 1.0], 0.3, 101, 64, 0.635
    c = systems.unit([0.0, 0.6, 0.8])
    ref = rt.get_ray_fan(pt, th, nt, wl, nphis=nph, center_ray=tuple(c))
    tdt = torch.float64 if dtype == C.RTPB_F64 else torch.float32
    out = torch.empty((nt * nph, 8), dtype=tdt, device=DEV)
    C.check(C.lib().rtpb_ray_fan(0, dtype, out.data_ptr(), _d3(pt), th, nt, nph, _d3(c), wl,
                                 torch.cuda.current_stream(DEV).cuda_stream))
    got = out.double().cpu().numpy()
    assert got.shape == ref.shape
    tol = 4e-16 if dtype == C.RTPB_F64 else 1.2e-7
    np.testing.assert_allclose(got[:, :6], ref[:, :6].astype(np.float32 if tdt == torch.float32 else np.float64),
                               rtol=0, atol=tol * 4)
    assert np.array_equal(got[:, 6:], ref[:, 6:].astype(np.float32).astype(np.float64) if tdt == torch.float32
                          else ref[:, 6:])


def test_device_trig_collimated_rays_close_to_reference_generator():
    pt, dmax, nd, nph, phi0, wl = [0.0, 1.0, -2.0], 3.0, 41, 16, 0.3, 0.5
    normal = systems.unit([np.sin(0.2), 0.0, np.cos(0.2)])
    ref = rt.get_collimated_rays(pt, dmax, nd, wl, nphis=nph, phi_start=phi0, normal=normal)
    out = torch.empty((nd * nph, 8), dtype=torch.float64, device=DEV)
    C.check(C.lib().rtpb_collimated_rays(0, C.RTPB_F64, out.data_ptr(), _d3(pt), dmax, nd, nph, phi0, _d3(normal), wl,
                                         torch.cuda.current_stream(DEV).cuda_stream))
    got = out.cpu().numpy()
    assert got.shape == ref.shape
    np.testing.assert_allclose(got, ref, rtol=0, atol=1e-14)
    assert np.array_equal(got[:, 3:], ref[:, 3:])            # directions, phase, wavelength: no trig


def test_shutdown_then_trace_again():
    system, rays, m0, m1 = systems.c1_plano_convex(rt, mat)
    before = system.ray_trace(rays, m0, m1)
    torch.cuda.synchronize()
    E.clear_plan_cache()                                      # plans must be destroyed first
    C.check(C.lib().rtpb_shutdown())
    after = system.ray_trace(rays, m0, m1)
    assert same_bits(after, before)
    x = torch.from_numpy(rays).to(DEV)
    assert same_bits(system.ray_trace(x, m0, m1).cpu().numpy(), before)


GEN_CASES = {   # tests/golden/make_golden.py: the reference's own generators (RT:45-161) on these arguments
    "fan": ("fan", ([1., 2., 3.], 0.3, 7, 0.5), dict(nphis=5, center_ray=(0, 0, 1))),
    "fan_tilted": ("fan", ([0., 0., 0.], 0.2, 5, 0.6), dict(nphis=3, center_ray=tuple(systems.unit([0.6, 0, 0.8])))),
    "coll": ("coll", ([0., 1., -2.], 3., 5, 0.5), dict(nphis=4, phi_start=0.3)),
    "coll_tilted": ("coll", ([0., 0., 0.], 2., 4, 0.5), dict(nphis=3, normal=[np.sin(0.2), 0, np.cos(0.2)])),
    "coll_y": ("coll", ([0., 0., 0.], 2., 3, 0.5), dict(nphis=2, normal=[0, 1, 0])),
}


@pytest.mark.parametrize("name", list(GEN_CASES))
def test_device_generators_bitwise_vs_reference_fixtures(name):
    """rtpb_ray_fan_tables / rtpb_collimated_rays_tables (through get_ray_fan / get_collimated_rays with
    device=) against the reference's own generator output in tests/golden/generators.npz: float64 bit for
    bit, float32 storage = the fixture rounded once; fans also as per-device phi-row shards."""
    import os
    from parity import GOLDEN
    ref = np.load(os.path.join(GOLDEN, "generators.npz"))[name]
    kind, args, kw = GEN_CASES[name]
    gen = rt.get_ray_fan if kind == "fan" else rt.get_collimated_rays
    got = gen(*args, **kw, device=DEV)
    assert got.dtype == torch.float64 and np.array_equal(got.cpu().numpy(), ref)
    got32 = gen(*args, **kw, device=DEV, dtype="float32")
    assert got32.dtype == torch.float32 and np.array_equal(got32.cpu().numpy(), ref.astype(np.float32))
    if kind == "fan":
        shards = gen(*args, **kw, devices=[0, 0, 0])
        assert np.array_equal(torch.cat([s.cpu() for s in shards]).numpy(), ref)


WL_CASES = {   # tests/golden/make_golden.py: per-ray wavelengths (RT:94, RT:115, RT:159); <name>_wl holds the array
    "fan_wl": ("fan", ([1., 2., 3.], 0.3, 7), dict(nphis=5)),
    "fan_wl3": ("fan", ([0., 0., -5.], 0.02, 11), dict(nphis=12)),
    "fan_wl1": ("fan", ([0., 0., 0.], 0.2, 5), dict(nphis=3, center_ray=tuple(systems.unit([0.6, 0, 0.8])))),
    "coll_wl": ("coll", ([0., 1., -2.], 3., 5), dict(nphis=4, phi_start=0.3)),
    "coll_wl_tilted": ("coll", ([0., 0., 0.], 2., 4), dict(nphis=3, normal=[np.sin(0.2), 0, np.cos(0.2)])),
}


@pytest.mark.parametrize("name", list(WL_CASES))
@pytest.mark.parametrize("wl_kind", ["numpy", "torch"])
def test_device_generators_per_ray_wavelengths_bitwise(name, wl_kind):
    """get_ray_fan / get_collimated_rays with one wavelength per ray (rtpb_*_tables_wl) against the
    reference's own output on the same arrays (generators.npz): float64 bit for bit, float32 storage = the
    fixture rounded once; the host generator gives the same bits; fans also as per-device phi-row shards."""
    import os
    from parity import GOLDEN
    d = np.load(os.path.join(GOLDEN, "generators.npz"))
    ref, wls = d[name], d[name + "_wl"]
    kind, args, kw = WL_CASES[name]
    gen = rt.get_ray_fan if kind == "fan" else rt.get_collimated_rays
    w = wls if wl_kind == "numpy" else torch.from_numpy(wls).to(DEV)
    got = gen(*args, w, **kw, device=DEV)
    assert got.dtype == torch.float64 and same_bits(got.cpu().numpy(), ref)
    got32 = gen(*args, w, **kw, device=DEV, dtype="float32")
    assert same_bits(got32.cpu().numpy(), ref.astype(np.float32))
    assert same_bits(gen(*args, wls, **kw), ref)                       # the host generator
    if kind == "fan":
        for devs in ([0, 0, 0], [0, 0]):
            shards = gen(*args, w, **kw, devices=devs)
            assert same_bits(torch.cat([s.cpu() for s in shards]).numpy(), ref)


def test_device_generators_reject_what_numpy_rejects():
    """A per-ray wavelength array of the wrong length fails as the reference's assignment does."""
    with pytest.raises(ValueError):
        rt.get_ray_fan([0., 0., 0.], 0.1, 5, np.ones(7), nphis=2, device=DEV)
    with pytest.raises((ValueError, RuntimeError)):
        rt.get_collimated_rays([0., 0., 0.], 1., 3, torch.ones(5, device=DEV), nphis=2, device=DEV)
