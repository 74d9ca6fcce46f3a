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
import warnings
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


# Only the C-ABI (gnn_*) leaves the library. Everything else -- the kernels' host stubs
# above all, which are weak template instantiations -- binds inside the library, so a
# second build of the same sources loaded into the process (build_variant, the A/B tools)
# launches its OWN kernels instead of being interposed by the first library's.
EXPORT_MAP = CSRC_DIR / "exports.map"


def _link_cmd(hipcc: str, out: Path, objs) -> list[str]:
    return [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-pthread",
            f"-Wl,--version-script={EXPORT_MAP}", "-o", str(out), *map(str, objs), "-ldl"]


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
    if force or procs or _stale(LIB_PATH, objs + [EXPORT_MAP]):
        tmp = LIB_PATH.with_suffix(".so.tmp")
        r = subprocess.run(_link_cmd(hipcc, tmp, objs), capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed:\n" + r.stdout + r.stderr)
        os.replace(tmp, LIB_PATH)
    # the plain-C example is optional: a missing C compiler or a failing example build warns
    # and leaves the library usable; tests/test_capi.py builds it explicitly
    try:
        build_examples(force)
    except (RuntimeError, OSError) as e:
        warnings.warn(f"examples/ not built: {e}", RuntimeWarning, stacklevel=2)
    return LIB_PATH


EXAMPLES_DIR = REPO_DIR / "examples"
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))


def build_examples(force: bool = False) -> list[Path]:
    """The plain-C callers under examples/ (gcc, linked against the library and the HIP
    runtime only), next to the library in lib/: the C-ABI exercised without Python."""
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        raise RuntimeError("no C compiler for examples/")
    outs = []
    for src in sorted(EXAMPLES_DIR.glob("*.c")):
        out = LIB_DIR / src.stem
        if force or _stale(out, [src, HEADER, LIB_PATH]):
            cmd = [cc, "-O2", "-std=c11", "-Wall", "-D__HIP_PLATFORM_AMD__",
                   f"-I{ROCM / 'include'}", str(src), "-o", str(out), f"-L{LIB_DIR}",
                   "-lgnn_mi355x", f"-L{ROCM / 'lib'}", "-lamdhip64", "-Wl,-rpath,$ORIGIN",
                   f"-Wl,-rpath,{ROCM / 'lib'}"]
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"{src.name} failed:\n" + r.stdout + r.stderr)
        outs.append(out)
    return outs


def build_variant(tag: str, defines: list[str], only: list[str] | None = None) -> Path:
    """Kernel-tuning build: the sources with extra ``-D`` flags, linked into
    ``lib/variants/libgnn_<tag>.so`` (same C-ABI; used by tools/*_ab.py only).
    ``only``: compile just these csrc file names with the defines and link the main
    build's objects for the rest (the main library must be built)."""
    if only:
        build()
    odir = OBJ_DIR / "variants" / tag
    odir.mkdir(parents=True, exist_ok=True)
    out = LIB_DIR / "variants" / f"libgnn_{tag}.so"
    out.parent.mkdir(parents=True, exist_ok=True)
    hipcc = _hipcc()
    headers = sorted(CSRC_DIR.glob("*.hpp")) + [HEADER]
    stamp = odir / "defines.txt"
    same = stamp.exists() and stamp.read_text() == "\n".join(defines)
    procs = [(src, subprocess.Popen(_compile_cmd(hipcc, src, odir / (src.stem + ".o"),
                                                 [f"-D{d}" for d in defines]),
                                    stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
             for src in sources()
             if (not only or src.name in only)
             and (not same or _stale(odir / (src.stem + ".o"), [src] + headers))]
    failed = [f"--- {src.name} ---\n{p.communicate()[0]}" for src, p in procs if p.wait() != 0]
    if failed:
        raise RuntimeError("hipcc failed:\n" + "\n".join(failed))
    stamp.write_text("\n".join(defines))
    objs = [(odir if not only or src.name in only else OBJ_DIR) / (src.stem + ".o")
            for src in sources()]
    r = subprocess.run(_link_cmd(hipcc, out, objs), capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("link failed:\n" + r.stdout + r.stderr)
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
