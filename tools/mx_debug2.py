"""Which (row, K range) does one A block scale act on?  Probe: scale 2 at one (row, block); explain the output
delta of every changed row by the K range (16-element granules) whose partial product matches it."""
import os, sys, itertools
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ergm_amd import ops  # noqa: E402

E4M3 = torch.float8_e4m3fn
dev = torch.device("cuda:0")
M, N, K = 64, 64, 128
g = torch.Generator().manual_seed(0)
A8 = (torch.randn(M, K, generator=g) * 3).to(E4M3).view(torch.uint8)
B8 = (torch.randn(N, K, generator=g) * 3).to(E4M3).view(torch.uint8)
Af = A8.view(E4M3).double()
Bf = B8.view(E4M3).double()
u = lambda r: torch.full((r, K // 32), 127, dtype=torch.uint8)  # noqa: E731
base = ops.gemm_mx(A8.to(dev), u(M).to(dev), B8.to(dev), u(N).to(dev)).double().cpu()
print("unit err", ((base - Af @ Bf.t()).norm() / base.norm()).item())
gran = [(Af[:, 16 * i:16 * i + 16] @ Bf[:, 16 * i:16 * i + 16].t()) for i in range(K // 16)]  # [M][N] each
for (r, j) in [(0, 0), (0, 1), (0, 2), (0, 3), (5, 0), (5, 2), (17, 1), (33, 3)]:
    sa = u(M).clone()
    sa[r, j] = 128
    o = ops.gemm_mx(A8.to(dev), sa.to(dev), B8.to(dev), u(N).to(dev)).double().cpu()
    d = o - base
    rows = (d.abs().amax(1) > 1e-3).nonzero().flatten().tolist()
    expl = []
    for rr in rows:
        best = None
        for a in range(K // 16):
            for b in range(a, K // 16):
                for subset in [list(range(a, b + 1))]:
                    pred = sum(gran[i][rr] for i in subset)
                    e = (pred - d[rr]).norm().item() / max(d[rr].norm().item(), 1e-9)
                    if best is None or e < best[0]:
                        best = (e, subset)
        # also try pairs of non-contiguous granules
        for i1, i2 in itertools.combinations(range(K // 16), 2):
            pred = gran[i1][rr] + gran[i2][rr]
            e = (pred - d[rr]).norm().item() / max(d[rr].norm().item(), 1e-9)
            if e < best[0]:
                best = (e, [i1, i2])
        expl.append((rr, [16 * i for i in best[1]], round(best[0], 4)))
    print(f"A scale (row {r}, block {j}) x2 -> rows {rows}; k16 granules: {expl}", flush=True)
