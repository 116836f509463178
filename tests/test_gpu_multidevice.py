"""GPU: device-resident multi-GPU paths in one process and systems longer than one fused
launch (> RTPB_MAX_SURFACES surfaces).  Rays are independent, so every sharded or segmented trace must be
BIT-IDENTICAL to the single-launch trace and to the NumPy oracle.  On a one-GPU box the shards share
device 0 (same code path: per-shard copies, launches and gathers); with more GPUs the same tests also
run across devices."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

import ray_trace_pb_amd.materials as mat  # noqa: E402
import ray_trace_pb_amd.raytrace as rt  # noqa: E402
from ray_trace_pb_amd import _capi as C  # noqa: E402
from oracle import rt_numpy as O  # noqa: E402
from serialize import material_to_dict, surface_to_dict  # noqa: E402
import systems  # noqa: E402
from parity import same_bits  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def oracle(system, m0, m1, rays):
    return O.ray_trace([surface_to_dict(s) for s in system.surfaces],
                       [material_to_dict(m) for m in [m0] + list(system.materials) + [m1]], rays)


def device_lists():
    n = torch.cuda.device_count()
    out = [[0, 0], [0, 0, 0]]
    if n > 1:
        out += [list(range(n)), [n - 1, 0]]
    return out


@pytest.mark.parametrize("devs", device_lists())
def test_torch_bundle_scattered_over_devices_is_bitwise_equal(devs):
    """torch bundle + devices: ray-index shards copied to each device, traced there, gathered back."""
    system, rays, m0, m1 = systems.stress(rt, mat)
    x = torch.from_numpy(rays).to(DEV)
    ref = system.ray_trace(x, m0, m1).cpu().numpy()
    assert same_bits(ref, oracle(system, m0, m1, rays))
    got = system.ray_trace(x, m0, m1, devices=devs)
    assert got.device == x.device and same_bits(got.cpu().numpy(), ref)
    parts = system.ray_trace(x, m0, m1, devices=devs, gather=False)
    assert isinstance(parts, list) and len(parts) == len(devs)
    for p, d, (a, b) in zip(parts, devs, rt.shard_bounds(x.shape[0], len(devs))):
        assert p.device.index == d and p.shape[1] == b - a
    assert same_bits(np.concatenate([p.cpu().numpy() for p in parts], axis=1), ref)
    # float32 storage, final plane, SoA
    f32 = system.ray_trace(x, m0, m1, devices=devs, dtype="float32", planes="final", layout="soa")
    assert same_bits(f32.cpu().numpy(), ref[-1:].astype(np.float32).transpose(0, 2, 1))


@pytest.mark.parametrize("devs", device_lists())
def test_per_device_fan_shards_traced_in_place(devs):
    """C4-style: the fan is generated as per-device shards (whole phi rows) and traced where it lives;
    the shards concatenate to the reference-style fan and their histories to the unsharded history."""
    system, m0, m1 = systems.c4_system(rt, mat), mat.Constant(systems.OPM_N1), mat.Vacuum()
    theta = 30 * np.pi / 180
    args = ([1e-3, 1e-3, 1e-3 * np.tan(theta)], np.arcsin(1.35 / systems.OPM_N1), 301, systems.OPM_WAVELENGTH)
    host = rt.get_ray_fan(*args, nphis=101)
    shards = rt.get_ray_fan(*args, nphis=101, devices=devs)
    assert [s.device.index for s in shards] == devs
    assert np.array_equal(np.concatenate([s.cpu().numpy() for s in shards]), host)
    hist = system.ray_trace(shards, m0, m1, dtype="float32")
    assert isinstance(hist, list) and all(h.device == s.device for h, s in zip(hist, shards))
    ref = oracle(system, m0, m1, host)
    assert same_bits(np.concatenate([h.cpu().numpy() for h in hist], axis=1), ref.astype(np.float32))


@pytest.mark.parametrize("storage", ["float64", "float32"])
def test_long_system_bitwise_vs_oracle(storage):
    """104 surfaces (209 planes): two fused segments (63 + 41 surfaces) continuing from the first
    segment's last plane; NumPy and torch paths, all / final / selected planes, float64 and float32
    storage, 3-D history input."""
    system = systems.long_system(rt, mat)
    S = len(system.surfaces)
    assert S > C.RTPB_MAX_SURFACES
    rays = systems.long_rays(4099)
    m0, m1 = mat.Vacuum(), mat.Vacuum()
    ref = oracle(system, m0, m1, rays)
    live = np.isfinite(ref[-1, :, 0]).sum()
    assert 0 < live < rays.shape[0]
    exp = ref if storage == "float64" else ref.astype(np.float32)
    got = system.ray_trace(rays, m0, m1, dtype=storage)
    assert got.shape == (2 * S + 1, rays.shape[0], 8) and same_bits(got, exp)
    x = torch.from_numpy(rays).to(DEV)
    assert same_bits(system.ray_trace(x, m0, m1, dtype=storage).cpu().numpy(), exp)
    sel = [0, 1, 125, 126, 127, 128, 200, 2 * S]
    assert same_bits(system.ray_trace(rays, m0, m1, dtype=storage, planes=sel), exp[sel])
    fin = system.ray_trace(x, m0, m1, dtype=storage, planes="final", layout="soa")
    assert same_bits(fin.cpu().numpy(), exp[-1:].transpose(0, 2, 1))
    h3 = np.stack((rays, rays))
    got3 = system.ray_trace(h3, m0, m1)
    assert same_bits(got3[2:], ref[1:])
    sharded = system.ray_trace(x, m0, m1, dtype=storage, devices=[0, 0])
    assert same_bits(sharded.cpu().numpy(), exp)
