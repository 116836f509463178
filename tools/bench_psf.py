"""PSF pipeline of scripts/2022_02_06_perfect_imaging_system_psf.py at the script's own size (51 z-planes,
101 x 51-ray fans, 3241^2 pupil grid): device trace + GPU griddata + pupil field + hipFFT, vs the same
pipeline with scipy griddata on the host (interp='host').  Reports seconds per z-plane.

    python tools/bench_psf.py [--nz 51] [--host-planes 3]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ray_trace_pb_amd.materials as mat  # noqa: E402
import ray_trace_pb_amd.raytrace as rt  # noqa: E402
from ray_trace_pb_amd import analysis  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nz", type=int, default=51)
    ap.add_argument("--host-planes", type=int, default=3)
    args = ap.parse_args()
    wavelength, n1, na, mag, ftl = 532e-6, 1.4, 1.35, 100, 200       # the script's physical data
    alpha = np.arcsin(na / n1)
    f1 = ftl / mag
    r1 = na * f1
    system = rt.System([rt.PerfectLens(f1, [0, 0, n1 * f1], [0, 0, 1], alpha),
                        rt.FlatSurface([0, 0, n1 * f1 + f1], [0, 0, 1], 4 * r1),
                        rt.PerfectLens(ftl, [0, 0, n1 * f1 + f1 + ftl], [0, 0, 1], na / mag),
                        rt.FlatSurface([0, 0, n1 * f1 + f1 + 2 * ftl], [0, 0, 1], r1)],
                       [mat.Vacuum(), mat.Vacuum(), mat.Vacuum()])
    zs = 1e-4 * np.arange(args.nz, dtype=float)
    zs -= zs.mean()
    srcs = [[0, 0, z] for z in zs]
    kw = dict(pupil_plane=4, pupil_radius=r1, grid_step=5e-3, device="cuda:0")
    analysis.pupil_psf(system, mat.Constant(n1), mat.Vacuum(), srcs[:1], wavelength, alpha, 101, 51, **kw,
                       as_numpy=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    psf, pupil, xs = analysis.pupil_psf(system, mat.Constant(n1), mat.Vacuum(), srcs, wavelength, alpha, 101, 51,
                                        **kw, as_numpy=False)
    torch.cuda.synchronize()
    t_gpu = time.perf_counter() - t0
    hp = srcs[:args.host_planes]
    t0 = time.perf_counter()
    psf_h, _, _ = analysis.pupil_psf(system, mat.Constant(n1), mat.Vacuum(), hp, wavelength, alpha, 101, 51, **kw,
                                     interp="host", as_numpy=False)
    torch.cuda.synchronize()
    t_host = time.perf_counter() - t0
    g = analysis.pupil_psf(system, mat.Constant(n1), mat.Vacuum(), hp, wavelength, alpha, 101, 51, **kw,
                           as_numpy=False)[0]
    diff = float((g - psf_h).abs().max())
    # the script's host FFT of one pupil plane (numpy), for scale
    e = np.exp(1j * np.random.default_rng(0).uniform(0, 1, (len(xs), len(xs))))
    t0 = time.perf_counter()
    np.fft.fftshift(np.fft.fft2(np.fft.ifftshift(e)))
    t_np_fft = time.perf_counter() - t0
    print(json.dumps({"z_planes": args.nz, "grid": len(xs), "rays_per_plane": 101 * 51,
                      "numpy_fft2_s_per_plane": t_np_fft,
                      "gpu_interp_s_per_plane": t_gpu / args.nz, "host_interp_s_per_plane": t_host / len(hp),
                      "speedup": (t_host / len(hp)) / (t_gpu / args.nz),
                      "max_abs_psf_diff_gpu_vs_host_interp": diff}))


if __name__ == "__main__":
    main()
