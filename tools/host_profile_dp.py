"""cProfile of the data-parallel step's host work (fake process group, one GPU): which Python / ctypes calls
the per-bucket exchange spends its time in.  Usage: python tools/host_profile_dp.py [N]"""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["ERGM_BENCH_FAKE_PG"] = sys.argv[1] if len(sys.argv) > 1 else "8"
import bench  # noqa: E402

sys.argv = ["bench.py", "--no-cpu-baseline", "--steps", "20", "--warmup", "3", "--no-gpu-only"]
cProfile.run("bench.main()", "/tmp/dp.prof")
p = pstats.Stats("/tmp/dp.prof")
p.sort_stats("tottime").print_stats(35)
