"""CPU: the fingerprint and key cache behind the optimistic table keys of the torch path
(ray_trace_pb_amd/_engine.py; GPU behaviour in tests/test_gpu_table_miss.py)."""
import numpy as np

import ray_trace_pb_amd.materials as mat
from ray_trace_pb_amd import _engine as E
import systems


def test_tabulated_materials_are_the_ones_without_a_native_lowering():
    cauchy = systems.cauchy_class(mat)()
    ms = [mat.Vacuum(), mat.Constant(1.4), mat.Nsf11(), mat.Ebaf11(), cauchy]
    assert E.tabulated(ms) == ms[3:]


def test_fingerprint_tracks_attributes_and_class():
    C1 = systems.cauchy_class(mat)
    a, b = C1(), C1()
    assert E.table_fingerprint([a]) == E.table_fingerprint([b])
    b.b = 0.005
    assert E.table_fingerprint([a]) != E.table_fingerprint([b])
    C2 = systems.cauchy_class(mat)                       # same code, another class object
    assert E.table_fingerprint([a]) != E.table_fingerprint([C2()])
    e1, e2 = mat.Ebaf11(), mat.Ebaf11()
    assert E.table_fingerprint([e1]) == E.table_fingerprint([e2])
    e2.params[3] = 0.0
    assert E.table_fingerprint([e1]) != E.table_fingerprint([e2])
    a.arr = np.arange(3.0)
    fa = E.table_fingerprint([a])
    a.arr[1] = 7.0
    assert E.table_fingerprint([a]) != fa


def test_unfingerprintable_material_is_never_cached():
    C1 = systems.cauchy_class(mat)
    m = C1()
    m.cb = lambda w: w                                    # arbitrary objects: no fingerprint
    assert E.table_fingerprint([m]) is None
    E.remember_keys(None, np.array([0.5]))
    assert E.previous_keys(None) is None


def test_key_cache_is_bounded_lru():
    E._KEYS.clear()
    for k in range(E._KEYS_MAX + 5):
        E.remember_keys(("k", k), np.array([float(k)]))
    assert len(E._KEYS) == E._KEYS_MAX
    assert E.previous_keys(("k", 0)) is None
    assert E.previous_keys(("k", E._KEYS_MAX + 4))[0] == E._KEYS_MAX + 4
    E._KEYS.clear()
