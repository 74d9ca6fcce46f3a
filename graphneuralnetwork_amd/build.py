"""Offline build of the gfx950 aggregation library (libgnn_mi355x.so).

Every ``csrc/*.hip`` file is compiled by ``hipcc --offload-arch=gfx950`` into
an object (in parallel), then linked into ONE shared library that exports the
C-ABI declared in ``include/gnn_mi355x.h``.  The library lands in-tree
(``graphneuralnetwork_amd/lib/``) so it travels with the repository snapshot to
the GPU box; it is git-ignored.  hipcc cross-compiles without a GPU.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
REPO_DIR = PKG_DIR.parent
CSRC_DIR = PKG_DIR / "csrc"
LIB_DIR = PKG_DIR / "lib"
OBJ_DIR = LIB_DIR / "obj"
LIB_NAME = "libgnn_mi355x.so"
LIB_PATH = LIB_DIR / LIB_NAME
HEADER = REPO_DIR / "include" / "gnn_mi355x.h"
ARCH = os.environ.get("GNN_OFFLOAD_ARCH", "gfx950")

HIPCC_FLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-fPIC",
    "-std=c++17",
    "-munsafe-fp-atomics",
    "-Wall",
    "-Wno-unused-function",
]


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found: the gfx950 library cannot be built")


def sources() -> list[Path]:
    """HIP sources (*.hip, device + host) and host-only C++ (*.cpp, the CPython-exact sampler)."""
    return sorted(CSRC_DIR.glob("*.hip")) + sorted(CSRC_DIR.glob("*.cpp"))


def _compile_cmd(hipcc: str, src: Path, obj: Path, extra=()) -> list[str]:
    if src.suffix == ".cpp":  # host-only translation unit: the system C++ compiler
        return ["g++", "-O3", "-fPIC", "-std=c++17", "-Wall", "-pthread", *extra, "-c", str(src),
                "-o", str(obj)]
    return [hipcc, *HIPCC_FLAGS, *extra, "-c", str(src), "-o", str(obj)]


def _stale(target: Path, deps: list[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def build(force: bool = False, verbose: bool = False) -> Path:
    """Compile (if stale) and return the path of libgnn_mi355x.so."""
    srcs = sources()
    headers = sorted(CSRC_DIR.glob("*.hpp")) + [HEADER]
    OBJ_DIR.mkdir(parents=True, exist_ok=True)
    hipcc = _hipcc()
    procs = []
    objs = []
    for src in srcs:
        obj = OBJ_DIR / (src.stem + ".o")
        objs.append(obj)
        if force or _stale(obj, [src] + headers):
            cmd = _compile_cmd(hipcc, src, obj)
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
            procs.append((src, subprocess.Popen(cmd, stdout=subprocess.PIPE,
                                                stderr=subprocess.STDOUT, text=True)))
    failed = []
    for src, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            failed.append(f"--- {src.name} ---\n{out}")
        elif verbose and out.strip():
            print(out, file=sys.stderr)
    if failed:
        raise RuntimeError("hipcc failed:\n" + "\n".join(failed))
    if force or procs or _stale(LIB_PATH, objs):
        tmp = LIB_PATH.with_suffix(".so.tmp")
        cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-pthread", "-o", str(tmp),
               *map(str, objs)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed:\n" + r.stdout + r.stderr)
        os.replace(tmp, LIB_PATH)
    return LIB_PATH


def build_variant(tag: str, defines: list[str]) -> Path:
    """Kernel-tuning build: every source with extra ``-D`` flags, linked into
    ``lib/variants/libgnn_<tag>.so`` (same C-ABI; used by tools/*_ab.py only)."""
    odir = OBJ_DIR / "variants" / tag
    odir.mkdir(parents=True, exist_ok=True)
    out = LIB_DIR / "variants" / f"libgnn_{tag}.so"
    out.parent.mkdir(parents=True, exist_ok=True)
    hipcc = _hipcc()
    procs = [(src, subprocess.Popen(_compile_cmd(hipcc, src, odir / (src.stem + ".o"),
                                                 [f"-D{d}" for d in defines]),
                                    stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
             for src in sources()]
    failed = [f"--- {src.name} ---\n{p.communicate()[0]}" for src, p in procs if p.wait() != 0]
    if failed:
        raise RuntimeError("hipcc failed:\n" + "\n".join(failed))
    r = subprocess.run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-pthread", "-o", str(out),
                        *(str(odir / (src.stem + ".o")) for src in sources())],
                       capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("link failed:\n" + r.stdout + r.stderr)
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
