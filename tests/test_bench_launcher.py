"""bench.py --gpus N without torchrun starts N rank processes itself (CPU
check of that launch path over gloo; the GPU ranks use the same code)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env=None):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True,
                          timeout=180, env=e)


def test_gpus_n_spawns_n_ranks():
    r = _run(["--gpus", "2", "--selftest-launcher"])
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout            # rank 0 alone prints the line
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["rank_sum"] == 1.0


def test_world_size_mismatch_fails():
    r = _run(["--gpus", "4", "--selftest-launcher"], env={"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode == 2
    assert "WORLD_SIZE=2" in r.stderr


def test_failing_rank_fails_the_launch():
    # an unknown flag makes every rank exit 2 in argparse; the launcher must
    # report it instead of hanging or returning 0
    sys.path.insert(0, ROOT)
    import bench
    rc = bench.launch_ranks(2, ["--no-such-flag"])
    assert rc != 0
