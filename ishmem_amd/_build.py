"""Build the native library in-tree: ishmem_amd/libishmem_amd.so (HIP, gfx950).

Plain hipcc invocations (no cmake / torch JIT) so the .so lives in the repo tree and travels to
the GPU box with the snapshot.  Rebuilds only when a source or header is newer than the output.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
INCLUDE = ROOT / "include"
BUILD = ROOT / "build" / "native"
LIB = PKG / "libishmem_amd.so"
# The same library with the runtime's test hooks compiled in (ISHMEM_TEST_PCI_BUS,
# ISHMEM_TEST_FLAGS_UNAVAILABLE; -DISHMEMI_TEST_HOOKS): loaded only by the GPU tests that emulate
# one PE per GPU on the one-GPU box (ISHMEM_AMD_LIB).  Shares every kernel object with LIB.
LIB_TESTHOOKS = PKG / "libishmem_amd_testhooks.so"

# (source, object stem, extra flags): kernels_op.hip is compiled once per reduction op so the
# ~350 kernel instantiations build in parallel.
SOURCES = [("kernels.hip", "kernels", []), ("runtime.cpp", "runtime", []),
           ("bootstrap.cpp", "bootstrap", []), ("kernels_coll.hip", "kernels_coll", [])] + [
    ("kernels_op.hip", f"kernels_op{op}", [f"-DISHMEMI_KOP={op}"]) for op in range(7)]
ARCH = os.environ.get("ISHMEM_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found: the ishmem_amd native library needs ROCm's hipcc")


def _deps() -> list[Path]:
    return sorted(list(CSRC.glob("*")) + list(INCLUDE.glob("*.h")))


def needs_build() -> bool:
    if not LIB.exists() or not LIB_TESTHOOKS.exists():
        return True
    t = min(LIB.stat().st_mtime, LIB_TESTHOOKS.stat().st_mtime)
    return any(p.stat().st_mtime > t for p in _deps())


def build(force: bool = False, verbose: bool = False, defines: list[str] | None = None,
          out: Path | None = None) -> Path:
    """Build the library (or, with `defines` / `out`, an A/B variant of it at `out`, objects
    under build/native/<out stem>; the product library is never replaced by a variant)."""
    lib = LIB if out is None else Path(out)
    if out is None and not force and not needs_build():
        return LIB
    hipcc = _hipcc()
    bdir = BUILD if out is None else BUILD / lib.stem
    bdir.mkdir(parents=True, exist_ok=True)
    lib.parent.mkdir(parents=True, exist_ok=True)
    common = ["-O3", "-std=c++20", "-fPIC", f"--offload-arch={ARCH}", f"-I{INCLUDE}", f"-I{CSRC}",
              "-Wall", "-Wno-unused-function", *[f"-D{d}" for d in (defines or [])]]
    objs = []
    procs = []
    sources = list(SOURCES)
    if out is None:
        sources.append(("runtime.cpp", "runtime_testhooks", ["-DISHMEMI_TEST_HOOKS=1"]))
    for src, stem, extra in sources:
        obj = bdir / (stem + ".o")
        objs.append(obj)
        cmd = [hipcc, *common, *extra, "-c", str(CSRC / src), "-o", str(obj)]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append((cmd, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
    for cmd, p in procs:
        out_, _ = p.communicate()
        if p.returncode != 0:
            raise RuntimeError(f"hipcc failed: {' '.join(cmd)}\n{out_.decode(errors='replace')}")

    def link(target: Path, objects: list[Path]) -> None:
        tmp = target.with_suffix(".so.tmp")
        cmd = [hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", str(tmp), *map(str, objects)]
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout.decode(errors='replace')}")
        os.replace(tmp, target)

    product = [o for o in objs if o.stem != "runtime_testhooks"]
    link(lib, product)
    if out is None:
        link(LIB_TESTHOOKS, [bdir / "runtime_testhooks.o" if o.stem == "runtime" else o for o in product])
    return lib


if __name__ == "__main__":
    # python -m ishmem_amd._build [--force] [--define NAME=V ... --out PATH]  (A/B variants)
    args = sys.argv[1:]
    defs = [args[i + 1] for i, a in enumerate(args) if a == "--define"]
    outp = args[args.index("--out") + 1] if "--out" in args else None
    print(build(force="--force" in args, verbose=True, defines=defs, out=Path(outp) if outp else None))
