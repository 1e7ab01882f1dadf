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

SOURCES = ["odd_k912.hip", "odd_k58.hip", "odd_bp.hip", "kernels.hip", "odd.hip", "wide.hip", "stripes.hip", "verify.hip", "md5.hip", "shardhash.cpp", "hbec.cpp", "ecutils.cpp", "plan.cpp", "hostpath.cpp", "batcher.cpp", "coalesce.cpp"]
HEADERS = ["kernels.h", "gf256.h", "internal.h", "gf_device.h", "pool.h", "odd_impl.h", "tuning.h", "xor_sched.h"]
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
          objdir: Path | None = None, extra=(), link=None) -> Path:
    """Build libhbec.so (or, for tuning experiments, a variant with extra -D
    definitions into `lib` / `objdir`; `extra` compile flags and a custom
    `link` command prefix are for the sanitizer build)."""
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
            jobs.append([hipcc, *_flags(defs), *extra, *lang, "-c", str(s), "-o", str(o)])

    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")

    with ThreadPoolExecutor(max_workers=min(4, max(1, len(jobs)))) as ex:
        list(ex.map(run, jobs))
    if force or jobs or _stale(lib, objs):
        if link:
            run([*link, "-o", str(lib), *map(str, objs)])
        else:
            run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(lib), *map(str, objs),
                 "-lpthread"])
        check_isa(lib)
    return lib


def check_isa(lib: Path) -> None:
    """Refuse a library whose record kernels touch an SGPR a hand-issued
    scalar load is still filling (isa_check.py; round 4's 12+4 fault).  The
    rejected library is moved aside, so nothing loads it."""
    from hummingbird_amd import isa_check

    n, bad = isa_check.check_library(lib, arch=ARCH)
    if n == 0 or bad:
        rej = Path(str(lib) + ".rejected")
        lib.replace(rej)
        detail = "; ".join(f"{k}: {v[:2]}" for k, v in list(bad.items())[:4]) or "no record kernels found"
        raise RuntimeError(f"{lib.name} refused ({len(bad)} of {n} record kernels read scalar-load "
                           f"destinations before their wait; moved to {rej.name}): {detail}")


ASAN_DIR = PKG / "build_asan"
ASAN_LIB = ASAN_DIR / "libhbec_asan.so"
ASAN_EXE = ASAN_DIR / "host_asan"


def build_asan(force: bool = False, verbose: bool = False) -> Path:
    """AddressSanitizer + UBSan build of the HOST code of libhbec (device
    code is not instrumented: every -fsanitize on the hipcc lines sits behind
    -Xarch_host) and of the C driver tests/native/host_asan.c.  Host-only
    sanitizers are the ones this pool runs (no GPU ASan / xnack)."""
    clang = "/opt/rocm/lib/llvm/bin/clang"
    san_host = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
                "-Xarch_host", "-fno-sanitize-recover=undefined", "-Xarch_host", "-fno-omit-frame-pointer",
                "-Xarch_host", "-g"]
    rocm_lib = "/opt/rocm/lib"
    link = [clang + "++", "-shared", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
            f"-L{rocm_lib}", "-lamdhip64", "-lpthread", f"-Wl,-rpath,{rocm_lib}"]
    lib = build(force=force, verbose=verbose, lib=ASAN_LIB, objdir=ASAN_DIR / "obj", extra=san_host, link=link)
    src = ROOT / "tests" / "native" / "host_asan.c"
    if force or _stale(ASAN_EXE, [src, lib, INCLUDE / "hbec.h"]):
        cmd = [clang, "-std=c11", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
               "-fno-omit-frame-pointer", f"-I{INCLUDE}", str(src), f"-L{ASAN_DIR}", "-lhbec_asan",
               f"-Wl,-rpath,{ASAN_DIR}", f"-Wl,-rpath,{rocm_lib}", "-lpthread", "-o", str(ASAN_EXE)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"clang failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return ASAN_EXE


if __name__ == "__main__":
    build(force="--force" in sys.argv)
