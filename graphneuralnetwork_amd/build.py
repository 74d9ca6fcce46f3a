"""Offline build of the gfx950 aggregation library (libgnn_mi355x.so).

Every ``csrc/*.hip`` file is compiled by ``hipcc --offload-arch=gfx950`` into
an object (in parallel), then linked into ONE shared library that exports the
C-ABI declared in ``include/gnn_mi355x.h``.  The library lands in-tree
(``graphneuralnetwork_amd/lib/``) so it travels with the repository snapshot to
the GPU box; it is git-ignored.  hipcc cross-compiles without a GPU.
"""
from __future__ import annotations

import hashlib
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


def _headers() -> list[Path]:
    return sorted(CSRC_DIR.glob("*.hpp")) + [HEADER]


def lib_source_stamp(defines=()) -> str:
    """sha256 (16 hex) of what the library is built from: every csrc source and header, the
    export map, include/gnn_mi355x.h, the compile flags and the -D defines. ``build()`` embeds
    it in the library (``gnn_build_stamp()``); ``_lib.load()`` refuses a library whose stamp
    differs from the tree it is loaded from (the binary tied to the tree)."""
    h = hashlib.sha256()
    h.update(" ".join([*HIPCC_FLAGS, *defines]).encode() + b"\0")
    for f in sources() + _headers() + [EXPORT_MAP]:
        h.update(f.name.encode() + b"\0" + f.read_bytes() + b"\0")
    return h.hexdigest()[:16]


def _object_digest(src: Path, extra=()) -> str:
    """Content hash of one object's inputs (its source, every header, its flags): objects are
    rebuilt when this changes, not by mtime (a snapshot copy resets mtimes)."""
    h = hashlib.sha256(" ".join([*HIPCC_FLAGS, *extra]).encode())
    for f in [src] + _headers():
        h.update(f.read_bytes())
    return h.hexdigest()


def _needs_compile(src: Path, obj: Path, extra=()) -> bool:
    sig = obj.with_suffix(".o.sha256")
    return not (obj.exists() and sig.exists() and sig.read_text() == _object_digest(src, extra))


def _compile_all(hipcc: str, jobs, verbose: bool = False) -> None:
    """jobs: (src, obj, extra defines). Compiles in parallel, records each object's digest."""
    procs = []
    for src, obj, extra in jobs:
        cmd = _compile_cmd(hipcc, src, obj, extra)
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append((src, obj, extra, subprocess.Popen(cmd, stdout=subprocess.PIPE,
                                                        stderr=subprocess.STDOUT, text=True)))
    failed = []
    for src, obj, extra, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            failed.append(f"--- {src.name} ---\n{out}")
            continue
        obj.with_suffix(".o.sha256").write_text(_object_digest(src, extra))
        if verbose and out.strip():
            print(out, file=sys.stderr)
    if failed:
        raise RuntimeError("hipcc failed:\n" + "\n".join(failed))


def _stamp_object(odir: Path, stamp: str, defines=()) -> Path:
    """build_stamp.o: ``const char* gnn_build_stamp(void)`` returning the source stamp (and,
    for a variant build, its defines), compiled by the system C compiler."""
    src = odir / "build_stamp.c"
    obj = odir / "build_stamp.o"
    text = ("/* generated by graphneuralnetwork_amd/build.py */\n"
            f"const char* gnn_build_stamp(void) {{ return \"{stamp}\"; }}\n"
            f"const char* gnn_build_defines(void) {{ return \"{' '.join(defines)}\"; }}\n")
    if not (src.exists() and obj.exists() and src.read_text() == text):
        src.write_text(text)
        r = subprocess.run(["gcc", "-O2", "-fPIC", "-c", str(src), "-o", str(obj)],
                           capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("build_stamp.c failed:\n" + r.stdout + r.stderr)
    return obj


def build(force: bool = False, verbose: bool = False) -> Path:
    """Compile (what changed) and return the path of libgnn_mi355x.so, whose embedded
    ``gnn_build_stamp()`` is ``lib_source_stamp()`` of this tree."""
    srcs = sources()
    OBJ_DIR.mkdir(parents=True, exist_ok=True)
    hipcc = _hipcc()
    objs = [OBJ_DIR / (src.stem + ".o") for src in srcs]
    jobs = [(src, obj, ()) for src, obj in zip(srcs, objs) if force or _needs_compile(src, obj)]
    _compile_all(hipcc, jobs, verbose)
    stamp = lib_source_stamp()
    stamp_file = LIB_PATH.with_suffix(".stamp")
    objs.append(_stamp_object(OBJ_DIR, stamp))
    if (force or jobs or not LIB_PATH.exists() or not stamp_file.exists()
            or stamp_file.read_text() != stamp):
        tmp = LIB_PATH.with_suffix(".so.tmp")
        r = subprocess.run(_link_cmd(hipcc, tmp, objs), capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed:\n" + r.stdout + r.stderr)
        os.replace(tmp, LIB_PATH)
        stamp_file.write_text(stamp)
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
    extra = tuple(f"-D{d}" for d in defines)
    _compile_all(hipcc, [(src, odir / (src.stem + ".o"), extra) for src in sources()
                         if (not only or src.name in only)
                         and _needs_compile(src, odir / (src.stem + ".o"), extra)])
    objs = [(odir if not only or src.name in only else OBJ_DIR) / (src.stem + ".o")
            for src in sources()]
    objs.append(_stamp_object(odir, lib_source_stamp(extra), extra))
    r = subprocess.run(_link_cmd(hipcc, out, objs), capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("link failed:\n" + r.stdout + r.stderr)
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
