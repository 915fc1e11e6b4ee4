"""bench.py's multi-GPU launch contract, rehearsed on CPU: `bench.py --gpus 2`
(outside torch.distributed.run) starts two ranks itself, both see world size
2, and rank 0's line reports n_gpus 2 and the gathered rows of both ranks'
windows (config E's final gather).  The --dry-run engine
writes stand-in rows instead of running the GPU path."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _run(args, timeout=300):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.pop("LOCAL_RANK", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd="/tmp", env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


def test_gpus_2_launches_two_ranks_and_gathers_both():
    steps, per_step = 2, 5
    line = _run(["--gpus", "2", "--dry-run", "--steps", str(steps), "--warmup", "0",
                 "--stream-step-windows", str(per_step)])
    per_rank = steps * per_step
    assert line["dry_run"] is True and line["value"] is None
    assert line["n_gpus"] == 2
    assert line["config"]["windows_per_gpu"] == per_rank
    par = line["parity"]
    assert par["gathered_windows"] == 2 * per_rank
    assert par["gathered_rows_equal_expected"] is True
    assert par["gathered_rank0_rows_equal_local"] is True
    assert par["gathered_all_status_ok"] is True
    # the N > 1 line carries the CPU leg (rank 0, after the GPU region) with a
    # per-core rate, and names its like-for-like N = 1 point
    cpu = line["cpu_baseline"]
    assert cpu is not None and cpu["value"] > 0 and cpu["unit"] == "windows/s"
    assert cpu["value_per_core"] > 0 and cpu["cores"] >= 1
    assert "--config E" in line["config"]["anchor"]


def test_gpus_3_uneven_world():
    line = _run(["--gpus", "3", "--dry-run", "--steps", "1", "--warmup", "0", "--stream-step-windows", "4"])
    assert line["n_gpus"] == 3
    assert line["parity"]["gathered_windows"] == 12
    assert line["parity"]["gathered_rows_equal_expected"] is True


def test_dry_run_rejects_other_configs():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run", "--config", "B"], cwd="/tmp",
                       env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode != 0


def test_busy_union():
    import bench
    s = np.array([0.0, 1.0, 5.0, 5.5], np.float32)
    e = np.array([2.0, 3.0, 6.0, 5.7], np.float32)
    assert abs(bench.busy_union_ms(s, e) - 4.0) < 1e-6
    assert bench.busy_union_ms(np.zeros(0), np.zeros(0)) == 0.0


def test_dry_rows_are_seed_functions():
    import bench
    a = bench.dry_rows(1, 10, 64)
    b = bench.dry_rows(6, 5, 64)
    for x, y in zip(a, b):
        assert np.array_equal(x[5:], y)
