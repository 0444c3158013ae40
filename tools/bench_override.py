"""bench.py with GEMM configuration overrides: python tools/bench_override.py M,N,K,al,bl,cfg,split [...] -- <bench args>
(ergm_gemm_set_override before the run; the bench line's roofline probe then times the overridden launch)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from ergm_amd import _lib as L  # noqa: E402

i = sys.argv.index("--") if "--" in sys.argv else len(sys.argv)
torch.cuda.init()  # the HIP runtime sees the device through torch's initialisation first
lib = L.load()
for spec in sys.argv[1:i]:
    M, N, K, al, bl, c, sp = (int(x) for x in spec.split(","))
    L.check(lib.ergm_gemm_set_override(M, N, K, al, bl, c, sp), "override")
sys.argv = ["bench.py"] + sys.argv[i + 1:]

bench.main()
