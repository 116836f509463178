"""Generate the golden vectors in tests/golden/*.npz from the REFERENCE implementation.

Run from anywhere inside this container (not on the GPU box -- /root/reference does not exist there):

    python tests/golden/make_golden.py [name,...]     # only the named recipes (no paraxial/generator files)
    python tests/golden/make_golden.py generators     # only generators.npz

The script re-launches itself in a child interpreter whose ``sys.path`` holds only
/root/reference/src (the reference's ``raytrace`` package) and this directory, with cwd=/tmp, so the
reference and this repository's drop-in ``raytrace`` alias can never be confused (SURVEY.md §7 hard
part 7).  The child builds each recipe of ``systems.py`` with the reference API, runs the reference's
``System.ray_trace`` (RT:641-661) and stores, per case, the input rays, the full returned history and
the serialised system.  Paraxial known answers (ray-transfer matrices, cardinal points, Seidel sums)
go to paraxial.json.  Only data is stored -- no reference source or bytecode.
"""
import json
import os
import subprocess
import sys
import warnings

HERE = os.path.dirname(os.path.abspath(__file__))
REF_SRC = "/root/reference/src"


def _child():
    import numpy as np
    import raytrace.raytrace as rt          # the REFERENCE (only REF_SRC is on the path)
    import raytrace.materials as mat
    assert os.path.abspath(rt.__file__).startswith(REF_SRC), rt.__file__
    import systems
    from serialize import system_to_json

    warnings.simplefilter("ignore")
    meta = {"numpy": np.__version__, "reference": "QI2lab/ray_trace_pb @ 2024_10_08"}

    only = [v for v in os.environ.get("RTPB_GOLDEN_ONLY", "").split(",") if v]
    if only == ["generators"]:
        _generators(np, rt, systems)
        return
    # float32 INPUT variants (<recipe>_f32in): the reference run on the recipe's rays rounded to
    # float32, i.e. what a caller handing it float32 arrays gets back (a float64 history)
    recipes = [(n, r, False) for n, r in systems.RECIPES.items()]
    recipes += [(n + "_f32in", systems.RECIPES[n], True) for n in systems.F32_INPUT_CASES]
    for name, recipe, f32in in recipes:
        if only and name not in only:
            continue
        system, rays, m_init, m_final = recipe(rt, mat)
        rays = np.asarray(rays, dtype=np.float32 if f32in else np.float64)
        hist = system.ray_trace(rays, m_init, m_final)
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"),
                            rays_in=rays,
                            history=np.asarray(hist, dtype=np.float64),
                            system_json=np.array(system_to_json(system, m_init, m_final)),
                            meta_json=np.array(json.dumps(meta)))
        print(f"{name:24s} surfaces={len(system.surfaces):2d} rays_in={rays.shape} history={hist.shape} "
              f"nan_rows_final={int(np.isnan(hist[-1]).any(axis=1).sum())}")
    if only:
        return

    # input-rank cases of System.ray_trace (RT:1175-1178: 1-D -> (1,1,8), 2-D -> (1,N,8), 3-D appended)
    system, rays, m_init, m_final = systems.c1_plano_convex(rt, mat, nrays=5)
    shapes = {"rays2": rays, "out2": system.ray_trace(rays, m_init, m_final),
              "rays1": rays[2], "out1": system.ray_trace(rays[2], m_init, m_final)}
    rays3 = np.stack((rays, rays + np.array([0, 0, -1, 0, 0, 0, 0, 0])), axis=0)
    shapes.update(rays3=rays3, out3=system.ray_trace(rays3, m_init, m_final))
    np.savez_compressed(os.path.join(HERE, "shapes.npz"),
                        system_json=np.array(system_to_json(system, m_init, m_final)), **shapes)

    # paraxial known answers
    par = {"meta": meta, "cases": []}
    for name in ("c1_plano_convex", "c2_achromat", "c3_relay", "c5_odt"):
        system, _, m_init, m_final = systems.RECIPES[name](rt, mat)
        for wl in (0.5876, 0.855):
            rtm = system.get_ray_transfer_matrix(wl, m_init, m_final)
            cp = system.get_cardinal_points(wl, m_init, m_final)
            par["cases"].append({"name": name, "wavelength": wl, "rtm": np.asarray(rtm).tolist(),
                                 "cardinal": [np.asarray(c, dtype=float).tolist() for c in cp],
                                 "auto_focus_paraxial_collimated":
                                     float(system.auto_focus(wl, m_init, m_final, mode="paraxial-collimated"))})
    # tests/rt_unittest.py:20-41 (Kidger 8.2.2 doublet) Seidel sums
    l1 = rt.Doublet(mat.Nsk11(), mat.Nsf19(), radius_crown=64.1, radius_flint=-183.685,
                    radius_interface=-43.249, thickness_crown=3.5, thickness_flint=1.5,
                    aperture_radius=10., input_collimated=True)
    kid = l1.concatenate(rt.FlatSurface([0, 0, 0], [0, 0, 1], 25.4), mat.Vacuum(), 10)
    kid.set_aperture_stop(0)
    ab = kid.seidel_third_order(0.5876, mat.Vacuum(), mat.Vacuum(), object_distance=np.inf,
                                object_angle=0.01746)
    par["kidger_seidel"] = np.asarray(ab).tolist()
    # ray-fan autofocus of C2 (calls ray_trace with 3 rays, RT:832-836)
    system, _, m_init, m_final = systems.RECIPES["c1_plano_convex"](rt, mat)
    par["c1_auto_focus_collimated"] = np.asarray(system.auto_focus(0.5, m_init, m_final, mode="collimated")).tolist()
    with open(os.path.join(HERE, "paraxial.json"), "w") as f:
        json.dump(par, f, indent=1)

    _generators(np, rt, systems)


def _generators(np, rt, systems):
    """Ray generators and analysis utilities (RT:45-353) -> generators.npz."""
    gens = {
        "fan": rt.get_ray_fan([1., 2., 3.], 0.3, 7, 0.5, nphis=5, center_ray=(0, 0, 1)),
        "fan_tilted": rt.get_ray_fan([0., 0., 0.], 0.2, 5, 0.6, nphis=3,
                                     center_ray=tuple(systems.unit([0.6, 0, 0.8]))),
        "coll": rt.get_collimated_rays([0., 1., -2.], 3., 5, 0.5, nphis=4, phi_start=0.3),
        "coll_tilted": rt.get_collimated_rays([0., 0., 0.], 2., 4, 0.5, nphis=3,
                                              normal=[np.sin(0.2), 0, np.cos(0.2)]),
        "coll_y": rt.get_collimated_rays([0., 0., 0.], 2., 3, 0.5, nphis=2, normal=[0, 1, 0]),
    }
    r1 = systems.stress_rays(64, seed=5)
    r2 = systems.stress_rays(64, seed=6)
    gens["intersect_in1"], gens["intersect_in2"] = r1, r2
    gens["intersect_out"] = rt.intersect_rays(r1, r2)
    fan = rt.get_ray_fan([0., 0., 0.], 0.1, 5, 0.5)
    gens["intersect_fan_out"] = rt.intersect_rays(fan[1], fan)
    ang, na = rt.ray_angle_about_axis(r1, np.array([0., 0., 1.]))
    gens["angle_out"], gens["angle_na"] = ang, na
    dists, near = rt.dist_pt2plane(r1[:, :3], np.array([0., 0.6, 0.8]), np.array([1., 2., 3.]))
    gens["dist_out"], gens["dist_near"] = dists, near
    # per-ray wavelengths: "either floating point or an array the same size as n_disps * nphis" (RT:115; the
    # fan's RT:94 is the same assignment); the arrays are stored beside the bundles as <case>_wl
    wl_cases = {
        "fan_wl": ("fan", ([1., 2., 3.], 0.3, 7, np.linspace(0.4, 0.8, 35)), {"nphis": 5}),
        "fan_wl3": ("fan", ([0., 0., -5.], 0.02, 11, np.tile([0.7065, 0.855, 1.015], 44)), {"nphis": 12}),
        "fan_wl1": ("fan", ([0., 0., 0.], 0.2, 5, np.array([0.55])), {"nphis": 3,
                                                                       "center_ray": tuple(systems.unit([0.6, 0, 0.8]))}),
        "coll_wl": ("coll", ([0., 1., -2.], 3., 5, np.linspace(0.45, 0.65, 20, dtype=np.float32)),
                    {"nphis": 4, "phi_start": 0.3}),
        "coll_wl_tilted": ("coll", ([0., 0., 0.], 2., 4, np.repeat([0.405, 0.785], 6)),
                           {"nphis": 3, "normal": [np.sin(0.2), 0, np.cos(0.2)]}),
    }
    for name, (kind, args, kw) in wl_cases.items():
        fn = rt.get_ray_fan if kind == "fan" else rt.get_collimated_rays
        gens[name] = fn(*args, **kw)
        gens[name + "_wl"] = np.asarray(args[3])
    np.savez_compressed(os.path.join(HERE, "generators.npz"), **gens)


if __name__ == "__main__":
    if os.environ.get("RTPB_GOLDEN_CHILD") == "1":
        _child()
    else:
        env = dict(os.environ, PYTHONPATH=f"{REF_SRC}:{HERE}", RTPB_GOLDEN_CHILD="1",
                   RTPB_GOLDEN_ONLY=sys.argv[1] if len(sys.argv) > 1 else "",
                   MPLBACKEND="Agg", PYTHONDONTWRITEBYTECODE="1")
        sys.exit(subprocess.run([sys.executable, os.path.abspath(__file__)], env=env, cwd="/tmp").returncode)
