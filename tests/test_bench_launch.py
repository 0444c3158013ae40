"""bench.py --gpus N launches its own N rank processes (no external torch.distributed.run): here the
ranks rendezvous over gloo on the CPU through the launcher's environment and report back."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(n, extra_env=None):
    env = dict(os.environ, ERGM_BENCH_LAUNCH_PROBE="1", OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    env.update(extra_env or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(n), "--steps", "1",
                           "--warmup", "0"], capture_output=True, text=True, env=env, timeout=300)


def test_bench_self_launches_ranks():
    r = _run(3)
    assert r.returncode == 0, r.stderr
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout          # only rank 0 prints
    rec = json.loads(lines[0])
    assert rec["world_size"] == 3 and rec["rank_sum"] == 0 + 1 + 2


def test_bench_rejects_world_mismatch():
    env = dict(os.environ, ERGM_BENCH_LAUNCH_PROBE="1", WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "4"], capture_output=True,
                       text=True, env=env, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr
