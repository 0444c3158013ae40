"""Dropout keep masks restated in numpy — TEST INFRASTRUCTURE ONLY (the checker, never the product).

The reference draws its dropout masks with torch's generator inside ``nn.Dropout``
(src/model.py:142,245,266,506); those bits are not reproducible outside torch, so the build defines
its masks as a pure function of (seed, forward number, site, element) — include/ergm_hip.h
``ergm_dropout`` — and parity is pinned by replaying exactly those masks through the CPU oracle
(``gpt2_oracle.forward(dropout=...)``).  This module is the independent restatement of that
function, so the GPU generator is itself checked bit for bit:

* Philox4x32-10 (Salmon, Moraes, Dror, Shaw, "Parallel random numbers: as easy as 1, 2, 3", SC'11;
  Random123 — not a dependency of the reference, the published algorithm), pinned by the Random123
  known-answer vectors (``KAT``);
* counter = {g mod 2^32, g >> 32, site, offset}, key = seed, g = row·ceil(cols/4) + col/4; element
  col takes word col mod 4 and is kept iff that word >= round(p·2^32).
"""
from __future__ import annotations

import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
MASK32 = np.uint64(0xFFFFFFFF)

# Random123 kat_vectors, philox4x32 with 10 rounds: (counter[4], key[2]) -> output[4]
KAT = [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF, 0xFFFFFFFF), (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised over numpy uint32 arrays (broadcasting); returns four uint32 arrays."""
    x = [np.asarray(v, dtype=np.uint32) for v in (c0, c1, c2, c3)]
    x = np.broadcast_arrays(*x)
    x = [v.copy() for v in x]
    k0, k1 = np.uint32(k0), np.uint32(k1)
    with np.errstate(over="ignore"):
        for _ in range(10):
            p0 = M0 * x[0].astype(np.uint64)
            p1 = M1 * x[2].astype(np.uint64)
            hi0, lo0 = (p0 >> np.uint64(32)).astype(np.uint32), (p0 & MASK32).astype(np.uint32)
            hi1, lo1 = (p1 >> np.uint64(32)).astype(np.uint32), (p1 & MASK32).astype(np.uint32)
            x = [hi1 ^ x[1] ^ k0, lo1, hi0 ^ x[3] ^ k1, lo0]
            k0 = np.uint32(k0 + W0)
            k1 = np.uint32(k1 + W1)
    return x


def keep_mask(seed: int, offset: int, site: int, p: float, rows: int, cols: int, row0: int = 0) -> np.ndarray:
    """bool [rows, cols]: the keep mask of ergm_dropout{seed, offset, site, p, row0} (ergm_hip.h)."""
    if p <= 0.0:
        return np.ones((rows, cols), dtype=bool)
    thresh = np.uint32(min(round(p * 4294967296.0), 4294967295))
    cols4 = (cols + 3) // 4
    r = np.arange(rows, dtype=np.uint64)[:, None] + np.uint64(row0)
    c = np.arange(cols, dtype=np.uint64)[None, :]
    g = r * np.uint64(cols4) + c // np.uint64(4)
    w = philox4x32_10((g & MASK32).astype(np.uint32), (g >> np.uint64(32)).astype(np.uint32), np.uint32(site),
                      np.uint32(offset), seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    words = np.stack(w, axis=-1)                       # [rows, cols, 4]
    pick = np.take_along_axis(words, (c % np.uint64(4)).astype(np.int64)[..., None].repeat(rows, 0), axis=-1)[..., 0]
    return pick >= thresh
