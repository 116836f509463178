"""Oracle traces of large fans in parallel host processes -- TEST INFRASTRUCTURE (the checker of the
full-size C5 tests, tests/test_gpu_c5_full.py).  A fan is split into whole phi rows
(oracle.rt_numpy.ray_fan_rows, bit-identical to slices of the whole fan), each piece traced by the NumPy
oracle in a spawned worker process (never forked from a process that has initialised the GPU), and the
final planes are concatenated in ray order."""
import multiprocessing as mp
import os

import numpy as np


def _final_rows(args):
    S, M, pt, theta, nt, wl, nph, r0, r1, step = args
    from oracle import rt_numpy as O
    out = np.empty(((r1 - r0) * nt, 8))
    for a in range(r0, r1, step):
        b = min(r1, a + step)
        rays = O.ray_fan_rows(pt, theta, nt, wl, nph, a, b)
        out[(a - r0) * nt:(b - r0) * nt] = O.ray_trace(S, M, rays)[-1]
    return out


def fan_final_plane(S, M, pt, theta, nt, wl, nph, procs=None, rows_per_piece=16):
    """Final plane of the oracle's trace of ray_fan(pt, theta, nt, wl, nphis=nph) through (S, M)."""
    if procs is None:
        procs = max(1, min(16, len(os.sched_getaffinity(0))))
    bounds = [(nph * k // procs, nph * (k + 1) // procs) for k in range(procs)]
    jobs = [(S, M, list(map(float, pt)), float(theta), int(nt), float(wl), int(nph), a, b, rows_per_piece)
            for a, b in bounds if b > a]
    env_old = os.environ.get("OMP_NUM_THREADS")
    os.environ["OMP_NUM_THREADS"] = "1"
    try:
        with mp.get_context("spawn").Pool(len(jobs)) as pool:
            parts = pool.map(_final_rows, jobs)
    finally:
        if env_old is None:
            os.environ.pop("OMP_NUM_THREADS", None)
        else:
            os.environ["OMP_NUM_THREADS"] = env_old
    return np.concatenate(parts)
