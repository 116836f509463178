"""World-size-2 gloo test (CPU) of the multi-process path: contiguous ray shards, no data-path
collective, and the optional all-gather that re-assembles the history.  Each rank computes its shard
with the CPU harness of the kernel arithmetic (test-only stand-in for the GPU)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp
from parity import same_bits  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, result_dir):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.dirname(here), here, os.path.join(here, "golden")]
    import torch.distributed as dist
    import ray_trace_pb_amd.materials as mat
    import ray_trace_pb_amd.raytrace as rt
    from ray_trace_pb_amd import _capi as C
    from ray_trace_pb_amd import _engine as E
    from ray_trace_pb_amd.distributed import shard_bounds, trace_sharded
    from native_harness import harness_trace
    import systems

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    system, rays, m0, m1 = systems.stress(rt, mat, nrays=1001)

    def cpu_trace(s, r, a, b):
        low = E.lower(s.surfaces, [a] + list(s.materials) + [b], lambda: np.unique(rays[:, 7]), C.RTPB_F64)
        return harness_trace(low, r)

    lo, hi, local = trace_sharded(system, rays, m0, m1, trace_fn=cpu_trace)
    assert (lo, hi) == shard_bounds(1001, rank, world)
    full = trace_sharded(system, rays, m0, m1, gather=True, trace_fn=cpu_trace)
    np.save(os.path.join(result_dir, f"full{rank}.npy"), full)
    np.save(os.path.join(result_dir, f"local{rank}.npy"), local)
    dist.destroy_process_group()


def test_two_rank_sharded_trace_equals_unsharded(tmp_path):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    import ray_trace_pb_amd.materials as mat
    import ray_trace_pb_amd.raytrace as rt
    from ray_trace_pb_amd import _capi as C
    from ray_trace_pb_amd import _engine as E
    from native_harness import harness_trace
    import systems
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    system, rays, m0, m1 = systems.stress(rt, mat, nrays=1001)
    low = E.lower(system.surfaces, [m0] + list(system.materials) + [m1], lambda: np.unique(rays[:, 7]), C.RTPB_F64)
    ref = harness_trace(low, rays)
    for r in range(world):
        assert same_bits(np.load(tmp_path / f"full{r}.npy"), ref)
    parts = [np.load(tmp_path / f"local{r}.npy") for r in range(world)]
    assert same_bits(np.concatenate(parts, axis=1), ref)
