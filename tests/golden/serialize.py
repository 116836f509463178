"""JSON (de)serialisation of optical systems, duck-typed so it works on both the reference's
objects (inside make_golden.py's subprocess) and this repository's drop-in objects.

A serialised surface records its class name and every attribute the trace reads (reference
RT:1035-1069 base attributes plus the subclass extras: ``normal`` RT:1320/1389/1576, ``radius``
RT:1445, ``focal_len``/``alpha`` RT:1574-1575).  A serialised material records its class name and
its dispersion coefficients (MAT:32-33 Sellmeier b/c, MAT:64 Constant ``_n``, MAT:134 Ebaf11
``params``) or, for the user subclass of ``systems.cauchy_class``, its own parameters.
"""
import json
import numpy as np


def _vec(v):
    return [float(x) for x in np.asarray(v, dtype=float).ravel()]


def surface_to_dict(s):
    d = {"type": type(s).__name__,
         "input_axis": _vec(s.input_axis), "output_axis": _vec(s.output_axis),
         "center": _vec(s.center), "paraxial_center": _vec(s.paraxial_center),
         "aperture_rad": float(s.aperture_rad)}
    if hasattr(s, "normal"):
        d["normal"] = _vec(s.normal)
    if hasattr(s, "radius"):
        d["radius"] = float(s.radius)
    if hasattr(s, "focal_len"):
        d["focal_len"] = float(s.focal_len)
        d["alpha"] = float(s.alpha)
    return d


def material_to_dict(m):
    name = type(m).__name__
    if name == "Cauchy":
        return {"type": name, "a": float(m.a), "b": float(m.b)}
    if name == "Constant":
        return {"type": name, "n": float(m._n)}
    if hasattr(m, "params"):
        return {"type": name, "params": [float(p) for p in m.params]}
    return {"type": name, "b": [float(m.b1), float(m.b2), float(m.b3)],
            "c": [float(m.c1), float(m.c2), float(m.c3)]}


def system_to_json(system, m_init, m_final):
    return json.dumps({"surfaces": [surface_to_dict(s) for s in system.surfaces],
                       "materials": [material_to_dict(m) for m in [m_init] + list(system.materials) + [m_final]]})


def material_from_dict(mat, d):
    """Build a material of module ``mat`` from its serialised form."""
    t = d["type"]
    if t == "Cauchy":
        from systems import cauchy_class
        return cauchy_class(mat)(d["a"], d["b"])
    if t == "Constant":
        return mat.Constant(d["n"])
    if hasattr(mat, t):
        m = getattr(mat, t)()
    else:
        m = mat.Material(d["b"], d["c"])
    return m


def surface_from_dict(rt, d):
    """Build a surface of module ``rt`` and overwrite its attributes with the serialised ones
    (so systems transformed by reverse()/concatenate() come back exactly)."""
    t = d["type"]
    if t in ("FlatSurface", "PlaneMirror"):
        s = getattr(rt, t)(d["center"], d["normal"], d["aperture_rad"])
    elif t == "SphericalSurface":
        s = rt.SphericalSurface(d["radius"], d["center"], d["aperture_rad"], input_axis=d["input_axis"])
    elif t == "PerfectLens":
        s = rt.PerfectLens(d["focal_len"], d["center"], d["normal"], d["alpha"])
    else:
        raise ValueError(f"unknown surface type {t}")
    s.input_axis = np.array(d["input_axis"])
    s.output_axis = np.array(d["output_axis"])
    s.center = np.array(d["center"])
    s.paraxial_center = np.array(d["paraxial_center"])
    s.aperture_rad = d["aperture_rad"]
    if "normal" in d:
        s.normal = np.array(d["normal"])
    return s


def system_from_json(rt, mat, text):
    spec = json.loads(text)
    surfaces = [surface_from_dict(rt, d) for d in spec["surfaces"]]
    mats = [material_from_dict(mat, d) for d in spec["materials"]]
    return rt.System(surfaces, mats[1:-1]), mats[0], mats[-1]
