"""bench.py's rank launch (CPU): `--gpus N` is the number of ranks the line reports.

The driver's scaling run calls `bench.py --gpus N` either under torch.distributed.run or bare.
Bare, bench.py must start N ranks itself (a fresh launcher child, before anything touches the
GPU) and every rank must see WORLD_SIZE == N; a box with fewer GPUs must fail loudly instead
of printing an `n_gpus: 1` line. `--dry-launch` runs the launch and the gloo group (barrier,
max over ranks) without a GPU.
"""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def _env(**kv):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                           "MASTER_PORT")}
    env.update(kv)
    return env


def _run(args, env=None, timeout=240):
    return subprocess.run([sys.executable, str(ROOT / "bench.py")] + args, capture_output=True, text=True,
                          env=env or _env(), timeout=timeout, cwd=str(ROOT))


def _line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_bare_gpus_2_starts_two_ranks():
    p = _run(["--gpus", "2", "--dry-launch"])
    assert p.returncode == 0, p.stderr[-2000:]
    line = _line(p.stdout)
    assert line["world"] == 2 and line["n_gpus"] == 2
    assert sorted(r["rank"] for r in line["ranks"]) == [0, 1]
    assert all(r["world"] == 2 for r in line["ranks"])
    assert sorted(r["local_rank"] for r in line["ranks"]) == [0, 1]
    assert line["max_over_ranks"] == 1.0


def test_bare_gpus_3_starts_three_ranks():
    p = _run(["--gpus", "3", "--dry-launch"])
    assert p.returncode == 0, p.stderr[-2000:]
    assert _line(p.stdout)["world"] == 3


def test_gpus_1_runs_in_process():
    p = _run(["--dry-launch"])
    assert p.returncode == 0, p.stderr[-2000:]
    line = _line(p.stdout)
    assert line["world"] == 1 and line["n_gpus"] == 1


def test_launcher_world_must_match_gpus():
    # a launcher that started one rank while --gpus says 2: refused before anything runs
    p = _run(["--gpus", "2", "--dry-launch"], env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"))
    assert p.returncode != 0
    assert "WORLD_SIZE=1" in p.stderr


def test_not_enough_gpus_fails_loudly():
    # no GPU in this container: --gpus 2 must not fall back to a one-GPU line
    p = _run(["--gpus", "2", "--steps", "1", "--warmup", "0"])
    assert p.returncode != 0
    assert "needs 2 GPUs" in p.stderr
    assert '"n_gpus"' not in p.stdout


def test_launcher_parent_stays_off_the_gpu():
    """the parent that starts the ranks counts GPUs from the KFD topology in
    sysfs, so it never opens /dev/kfd nor loads the HIP runtime before its ranks start (it
    reports what it holds, from /proc/self)."""
    p = _run(["--gpus", "2", "--dry-launch"])
    assert p.returncode == 0, p.stderr[-2000:]
    assert "bench.py launcher: /dev/kfd open: no; HIP runtime loaded: no" in p.stderr, p.stderr[-2000:]


def test_gpu_count_from_sysfs():
    sys.path.insert(0, str(ROOT))
    import bench

    n = bench.gpu_count_sysfs()
    assert n >= 0
    old = os.environ.get("HIP_VISIBLE_DEVICES")
    os.environ["HIP_VISIBLE_DEVICES"] = "0"
    try:
        assert bench.gpu_count_sysfs() == min(n, 1)
    finally:
        if old is None:
            del os.environ["HIP_VISIBLE_DEVICES"]
        else:
            os.environ["HIP_VISIBLE_DEVICES"] = old
