"""Build libhbec.so in-tree for gfx950 with hipcc (no JIT cache, no cmake).

    python -m hummingbird_amd.build [--force]

Objects go to hummingbird_amd/build/, the shared library to
hummingbird_amd/libhbec.so (git-ignored, but shipped to the GPU box by gpurun).
"""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
OBJ = PKG / "build"
LIB = PKG / "libhbec.so"
ROOT = PKG.parent
INCLUDE = ROOT / "include"

SOURCES = ["kernels.hip", "stripes.hip", "verify.hip", "md5.hip", "shardhash.cpp", "hbec.cpp", "ecutils.cpp", "plan.cpp", "hostpath.cpp", "batcher.cpp"]
HEADERS = ["kernels.h", "gf256.h", "internal.h", "gf_device.h", "pool.h"]
ARCH = os.environ.get("HBEC_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.isabs(c) and os.path.exists(c) or not os.path.isabs(c)):
            return c
    return "hipcc"


def _flags(extra_defs=()) -> list[str]:
    f = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function",
         f"-I{INCLUDE}", f"-I{CSRC}"]
    f += [f"-D{d}" for d in extra_defs]
    return f


def _stale(target: Path, deps: list[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def build(force: bool = False, verbose: bool = True, defs=(), lib: Path | None = None,
          objdir: Path | None = None) -> Path:
    """Build libhbec.so (or, for tuning experiments, a variant with extra -D
    definitions into `lib` / `objdir`)."""
    lib = Path(lib) if lib else LIB
    objdir = Path(objdir) if objdir else OBJ
    objdir.mkdir(parents=True, exist_ok=True)
    hipcc = _hipcc()
    hdrs = [CSRC / h for h in HEADERS] + [INCLUDE / "hbec.h"]
    jobs = []
    objs = []
    for src in SOURCES:
        s = CSRC / src
        o = objdir / (src.rsplit(".", 1)[0] + ".o")
        objs.append(o)
        if force or _stale(o, [s] + hdrs):
            lang = ["-x", "hip"] if src.endswith(".hip") else []
            jobs.append([hipcc, *_flags(defs), *lang, "-c", str(s), "-o", str(o)])

    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")

    with ThreadPoolExecutor(max_workers=min(4, max(1, len(jobs)))) as ex:
        list(ex.map(run, jobs))
    if force or jobs or _stale(lib, objs):
        run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(lib), *map(str, objs),
             "-lpthread"])
    return lib


if __name__ == "__main__":
    build(force="--force" in sys.argv)
