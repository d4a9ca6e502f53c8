"""Builds the in-tree HIP library `beast_amd/libbeast_pmd.so` for gfx950.

hipcc compiles each translation unit under csrc/ (in parallel) and links one
shared library exporting the C ABI of include/beast_pmd.h.  The library is
built in-tree so it travels to the GPU box with the repository snapshot.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "_build")
LIB = os.path.join(HERE, "libbeast_pmd.so")
SYNTH = os.path.join(HERE, "libbpmd_synth.so")
ARCH = os.environ.get("BPMD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CXXFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
            "-munsafe-fp-atomics"]


# Machine scheduler per translation unit (LLVM AMDGPU -amdgpu-sched-strategy),
# measured interleaved on one MI355X (profiles/r06v_ab_sched_strategy.log):
# the lane decoder (issue-bound, dependent LDS lookups) gains from
# iterative-ilp -- C2 189.3 -> 191.2 GiB/s, inflate_lane3_kernel 1.305 -> 1.290
# ms, C5 own / Beast inflate +1.5 / +2 % -- and the deflate parse from max-ilp
# -- C3 52.6 -> 54.1, C4 30.9 -> 31.4 GiB/s.  Same results bit for bit.
SRC_FLAGS = {
    "pmd_inflate_lane3.hip": ["-mllvm", "-amdgpu-sched-strategy=iterative-ilp"],
    "pmd_deflate.hip": ["-mllvm", "-amdgpu-sched-strategy=max-ilp"],
}


def _sources():
    return sorted(f for f in os.listdir(CSRC) if f.endswith(".hip"))


def _headers_mtime():
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    hs.append(os.path.join(HERE, "..", "include", "beast_pmd.h"))
    return max(os.path.getmtime(h) for h in hs if os.path.exists(h))


def _compile(src: str, hmt: float, bdir: str = BUILD, extra=()) -> str:
    obj = os.path.join(bdir, src.replace(".hip", ".o"))
    s = os.path.join(CSRC, src)
    if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(s), hmt):
        return obj
    cmd = [HIPCC, *CXXFLAGS, *SRC_FLAGS.get(src, []), *extra, "-c", s, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
    return obj


def build(verbose: bool = False, variant: str = "") -> str:
    """variant "" = the product library; "prof" = diagnostic build with
    per-phase cycle counters (libbeast_pmd_prof.so, never loaded by default)."""
    bdir = BUILD + (f"_{variant}" if variant else "")
    lib = LIB.replace(".so", f"_{variant}.so") if variant else LIB
    extra = ("-DBPMD_PROF",) if variant == "prof" else ()
    # experiment variants: BPMD_EXTRA_FLAGS="-DBPMD_RING=8192 ..." python build.py <name>
    if variant and variant != "prof":
        extra = tuple(os.environ.get("BPMD_EXTRA_FLAGS", "").split())
    os.makedirs(bdir, exist_ok=True)
    hmt = _headers_mtime()
    srcs = _sources()
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(lambda s: _compile(s, hmt, bdir, extra), srcs))
    newest = max(os.path.getmtime(o) for o in objs)
    if not os.path.exists(lib) or os.path.getmtime(lib) < newest:
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib, *objs]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
    synth_src = os.path.join(CSRC, "synth.c")
    if not os.path.exists(SYNTH) or os.path.getmtime(SYNTH) < os.path.getmtime(synth_src):
        subprocess.run(["gcc", "-O2", "-fPIC", "-shared", "-o", SYNTH, synth_src, "-lm"], check=True)
    if verbose:
        print("built", lib)
    return lib


if __name__ == "__main__":
    build(verbose=True, variant=sys.argv[1] if len(sys.argv) > 1 else "")
    sys.exit(0)
