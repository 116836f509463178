"""bench.py contract on the CPU: the roofline object's fields and the algorithmic-byte accounting of the
BASELINE configs (16 w (S+1) bytes per ray of a full history).
The timed run itself needs a GPU (driver / gpurun)."""
import types

import bench


def test_c3_workload_size_and_bytes():
    nt, nph = bench.C3_FAN
    rays = 5 * nt * nph                                  # 5 field points x get_ray_fan(h, 1 deg, 3163, nphis=3162)
    assert rays == 50_007_030
    S, planes, w = 9, 19, 4
    contract = 16 * w * (S + 1)                          # one float32 input record + 19 float32 planes
    assert contract == 640 == 8 * w * (1 + planes)
    physical = 8 * 8 + planes * 8 * w                    # the input is read as float64
    assert physical == 672
    assert rays * physical == 33_604_724_160             # physical bytes per launch (PMC traffic: +0.0 %)
    assert rays * contract == 32_004_499_200


def test_c4_c5_sizes():
    nt, nph = bench.C4_FAN
    assert nt * nph == 100_010_000
    assert 16 * 4 * (11 + 1) * nt * nph == 76_807_680_000      # contract bytes of the 23-plane float32 history
    assert 64 * 7 * bench.C5_FAN[0] * bench.C5_FAN[1] == 4_480_629_888


def test_roofline_object_fields():
    wl = types.SimpleNamespace(alg_bytes=32_004_499_200, bytes_per_ray=640, S=9, phys_bytes=33_604_724_160,
                               phys_bytes_per_ray=672)
    r = bench.roofline(wl, 6.2, traffic=3.36e10, traffic_note=None, fill=6800.0, copy=4700.0)
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == bench.HBM_PEAK_GBS
    assert abs(r["achieved"] - 32_004_499_200 / 6.2e-3 / 1e9) < 1e-6
    assert abs(r["frac"] - r["achieved"] / 8000.0) < 1e-12
    assert abs(r["achieved_physical"] - 33_604_724_160 / 6.2e-3 / 1e9) < 1e-6
    assert abs(r["frac_of_output_fill"] - r["achieved_physical"] / 6800.0) < 1e-12
    assert r["torch_copy_GBps"] == 4700.0
    assert "torch_copy_GBps" not in bench.roofline(wl, 6.2)


def test_launcher_argv_runs_this_script_as_n_ranks():
    """`python bench.py --gpus N` outside torchrun starts torch.distributed.run on itself as a child process."""
    import os
    import sys
    argv = ["--gpus", "8", "--steps", "5", "--warmup", "2"]
    cmd = bench.launcher_argv(8, argv, 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29555" in cmd
    script = cmd.index(os.path.abspath(bench.__file__))
    assert cmd[script + 1:] == argv                     # the same arguments reach every rank


def test_world_size_checks_fail_loudly():
    import pytest
    args = types.SimpleNamespace(gpus=4, oversubscribe=False)
    with pytest.raises(SystemExit, match="WORLD_SIZE=2"):
        bench.check_world(args, 2, 8)                    # --gpus 4 under a 2-rank torchrun
    with pytest.raises(SystemExit, match="only 2 GPU"):
        bench.check_world(args, 4, 2)                    # more ranks than visible GPUs
    bench.check_world(args, 4, 8)
    bench.check_world(types.SimpleNamespace(gpus=4, oversubscribe=True), 4, 1)   # rehearsal on a shared GPU


def test_bench_gpus_n_without_gpus_fails_before_launching():
    """No GPU visible (this container): `bench.py --gpus 2` refuses before starting any rank.  On a host with
    two or more GPUs the command would start a real 2-rank benchmark, so the test does not apply there."""
    import os
    import subprocess
    import sys
    import pytest
    import torch
    if torch.cuda.device_count() >= 2:           # counts devices without initialising them on this image
        pytest.skip("two or more GPUs visible: bench.py --gpus 2 would run the benchmark")
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, bench.__file__, "--gpus", "2", "--steps", "1"], capture_output=True,
                       text=True, env=env, timeout=300)
    assert r.returncode != 0
    assert "GPU(s) visible" in r.stderr
    assert r.stdout.strip() == ""


def test_strong_scaling_fields():
    """configs.c4 / configs.c5 of an N > 1 line carry their own t1 (rank 0 alone, same job) and efficiency
    t1 / (N tN)."""
    r = bench.strong_scaling(13.5, 1.8, 8)
    assert r["t1_ms"] == 13.5 and r["tN_ms"] == 1.8
    assert abs(r["speedup"] - 7.5) < 1e-12
    assert abs(r["scaling_efficiency"] - 13.5 / (8 * 1.8)) < 1e-12
    assert abs(bench.strong_scaling(10.0, 5.0, 2)["scaling_efficiency"] - 1.0) < 1e-12
