"""cProfile of the data-parallel step's host work in the bench's timed loop (fake process group, one GPU):
which Python / ctypes calls the per-bucket exchange spends its time in.  Usage: python tools/host_profile_dp.py [N]
(N = fake world size; 1 = the single-process step)."""
import os
import pstats
import subprocess
import sys

here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
n = sys.argv[1] if len(sys.argv) > 1 else "8"
env = dict(os.environ, ERGM_BENCH_CPROFILE="/tmp/dp.prof")
if n != "1":
    env["ERGM_BENCH_FAKE_PG"] = n
subprocess.run([sys.executable, os.path.join(here, "bench.py"), "--no-cpu-baseline", "--steps", "20", "--warmup", "3",
                "--no-gpu-only"], env=env, check=True, stdout=subprocess.DEVNULL)
p = pstats.Stats("/tmp/dp.prof")
p.sort_stats("tottime").print_stats(25)
print("==== backward (autograd's thread: native stages + data-parallel exchange) ====")
q = pstats.Stats("/tmp/dp.prof.bwd")
q.sort_stats("tottime").print_stats(45)
q.sort_stats("cumulative").print_stats(30)
