"""rtpb_distinct_keys (include/rtpb.h): the distinct wavelengths of a device-resident bundle, the keys at
which RTPB_TABLE materials (Ebaf11, user Material.n) are evaluated.  Must equal np.unique of the column
(NaN collapsed and last), for float64 / float32, strided / contiguous columns; more keys than
DISTINCT_MAX_KEYS fall back to a sort with the same answer."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from ray_trace_pb_amd import _capi as C  # noqa: E402
from ray_trace_pb_amd import _engine as E  # noqa: E402
from parity import same_bits  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _ref(col):
    return np.unique(np.asarray(col, dtype=np.float64))


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_one_colour_and_mixed_bundles(dtype):
    rng = np.random.default_rng(3)
    n = 1_000_003
    rays = np.zeros((n, 8))
    rays[:, 7] = 0.635
    x = torch.from_numpy(rays).to(DEV, dtype)
    one = E._distinct_device(x[:, 7])
    assert one.size == 1 and np.array_equal(one, _ref(x[:, 7].cpu().numpy()))
    wls = np.array([0.405, 0.465, 0.488, 0.532, 0.561, 0.635, 0.785, 1e-3, 3.0])
    rays[:, 7] = wls[rng.integers(0, wls.size, n)]
    rays[rng.integers(0, n, 50), 7] = np.nan
    rays[rng.integers(0, n, 5), 7] = np.inf
    x = torch.from_numpy(rays).to(DEV, dtype)
    got = E._distinct_device(x[:, 7])
    exp = _ref(x[:, 7].cpu().numpy())
    assert got.shape == exp.shape and same_bits(got, exp)
    assert np.isnan(got[-1]) and np.isnan(got).sum() == 1
    # contiguous column, and the public entry point
    col = x[:, 7].contiguous()
    assert same_bits(E.distinct_wavelengths(col), exp)


def test_many_keys_fall_back_to_sort():
    rng = np.random.default_rng(4)
    col = torch.from_numpy(rng.uniform(0.4, 1.6, 200_000)).to(DEV)
    assert E._distinct_device(col) is None
    got = E.distinct_wavelengths(col)
    assert np.array_equal(got, _ref(col.cpu().numpy()))
    exact = torch.from_numpy(np.linspace(0.4, 1.6, E.DISTINCT_MAX_KEYS)).to(DEV)
    assert np.array_equal(E._distinct_device(exact), _ref(exact.cpu().numpy()))
    over = torch.from_numpy(np.linspace(0.4, 1.6, E.DISTINCT_MAX_KEYS + 1)).to(DEV)
    assert E._distinct_device(over) is None


def test_empty_and_errors():
    col = torch.zeros(0, dtype=torch.float64, device=DEV)
    assert E._distinct_device(col).size == 0
    lib = C.lib()
    ws = torch.empty(16, dtype=torch.int64, device=DEV)
    assert lib.rtpb_distinct_keys(0, ws.data_ptr(), C.RTPB_F64, 4, 1, ws.data_ptr(), 12, 4, ws.data_ptr(), None) != 0
    assert lib.rtpb_distinct_keys(0, ws.data_ptr(), C.RTPB_F64, 4, 1, ws.data_ptr(), 8, 5, ws.data_ptr(), None) != 0
