"""Build libergm_hip.so (gfx950) in-tree with hipcc.

Each source compiles to an object under ``build/`` in parallel; objects are rebuilt when the source
or any header under ``ergm_amd/csrc`` / ``include`` is newer.  The shared library lands next to this
file so it travels with the repo snapshot to the GPU box.
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(REPO, "include")
BUILD = os.path.join(REPO, "build")
LIB = os.path.join(HERE, "libergm_hip.so")
ARCH = os.environ.get("ERGM_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
SOURCES = ["abi.cpp", "gemm.hip", "attention.hip", "norm.hip", "embed.hip", "xent.hip", "adamw.hip", "quant.hip", "dropout.hip", "model.cpp"]
# -packed-fp32-ops: no v_pk_{add,mul,fma}_f32 in device code.  On gfx950 (ROCm 7.2) a packed FP32 instruction running
# while another wave of the same CU issues MFMAs can return a wrong low half in lanes 48-63 (the last quarter-wave):
# tools/adamw_hazard.hip measured ~1e-3 of the AdamW pass's words wrong beside MFMA waves, 0 alone and 0 without packed
# FP32.  Every kernel here can share a CU with a GEMM, so none may use them.  The host pass
# warns that it does not know the feature and ignores it.
DEVICE_FEATURES = ["-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"]
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", INCLUDE, "-Wall", "-Wno-unused-function",
         "-Wno-unused-variable", *DEVICE_FEATURES]


def _headers_mtime() -> float:
    m = 0.0
    for d in (CSRC, INCLUDE):
        for f in os.listdir(d):
            if f.endswith((".h", ".hpp")):
                m = max(m, os.path.getmtime(os.path.join(d, f)))
    return m


def _compile(src: str, hdr_m: float, verbose: bool) -> str:
    path = os.path.join(CSRC, src)
    obj = os.path.join(BUILD, src + ".o")
    if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(path), hdr_m):
        return obj
    cmd = [HIPCC, *FLAGS, "-c", path, "-o", obj]
    if src.endswith(".cpp"):
        cmd = [HIPCC, "-x", "hip", *FLAGS, "-c", path, "-o", obj]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    return obj


def _flags_stamp() -> float:
    """mtime of build/flags.txt, rewritten (forcing every object to rebuild) when the compile flags change."""
    stamp = os.path.join(BUILD, "flags.txt")
    want = " ".join([HIPCC, *FLAGS])
    if not os.path.exists(stamp) or open(stamp).read() != want:
        with open(stamp, "w") as f:
            f.write(want)
    return os.path.getmtime(stamp)


def build(verbose: bool = False, jobs: int = 8) -> str:
    os.makedirs(BUILD, exist_ok=True)
    hdr_m = max(_headers_mtime(), _flags_stamp())
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, hdr_m, verbose), SOURCES))
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB, *objs]
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    return LIB


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
