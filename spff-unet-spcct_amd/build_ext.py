"""Build libspff_hip.so (all HIP translation units, gfx950) in-tree.

    python spff-unet-spcct_amd/build_ext.py [--force]

Objects are compiled in parallel with hipcc, then linked into
``spff-unet-spcct_amd/innovative3D/_lib/libspff_hip.so``.  Rebuilds only when
the sha256 of the sources, headers and flags differs from the one recorded
beside the library at its build (``libspff_hip.build.json``; bench.py reports
both digests, so a stale binary cannot ship unnoticed).
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import json
import os
import pathlib
import shutil
import subprocess
import sys

PKG = pathlib.Path(__file__).resolve().parent
ROOT = PKG.parent
CSRC = PKG / "csrc"
INC = ROOT / "include"
OUT_DIR = PKG / "innovative3D" / "_lib"
LIB = OUT_DIR / "libspff_hip.so"
OBJ_DIR = PKG / "build" / "obj"
ARCH = os.environ.get("SPFF_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", f"-I{INC}", f"-I{CSRC}",
         "-Wno-unused-result"]


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm toolchain required to build libspff_hip.so)")


def sources():
    return sorted(CSRC.glob("*.hip"))


STAMP = OUT_DIR / "libspff_hip.build.json"


def _portable_flags():
    """the compile flags without the (checkout-dependent) include paths"""
    return [f for f in FLAGS if not f.startswith("-I")]


def source_digest() -> str:
    """sha256 over every translation unit, header and the compile flags"""
    h = hashlib.sha256(" ".join(_portable_flags()).encode())
    for p in sorted(list(sources()) + list(CSRC.glob("*.h")) + list(INC.glob("*.h"))):
        h.update(p.name.encode())
        h.update(p.read_bytes())
    return h.hexdigest()


def build_record() -> dict:
    """{"lib_sources_sha256": digest the library was built from (None: unknown),
    "tree_sources_sha256": digest of the sources now, "fresh": equal}"""
    built = None
    try:
        built = json.loads(STAMP.read_text()).get("sources_sha256")
    except Exception:
        pass
    now = source_digest()
    return {"lib": str(LIB.relative_to(ROOT)), "lib_sources_sha256": built,
            "tree_sources_sha256": now, "fresh": bool(LIB.exists() and built == now)}


def _stale() -> bool:
    return not build_record()["fresh"]


def build(force: bool = False, verbose: bool = True) -> pathlib.Path:
    if not force and not _stale():
        return LIB
    hipcc = _hipcc()
    OBJ_DIR.mkdir(parents=True, exist_ok=True)
    OUT_DIR.mkdir(parents=True, exist_ok=True)

    def compile_one(src: pathlib.Path):
        obj = OBJ_DIR / (src.stem + ".o")
        cmd = [hipcc, *FLAGS, "-c", str(src), "-o", str(obj)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src.name}:\n{r.stderr[-4000:]}")
        return obj

    jobs = min(8, max(1, len(sources())))
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(compile_one, sources()))
    tmp = LIB.with_suffix(".so.tmp")
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp), *map(str, objs)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr[-4000:]}")
    os.replace(tmp, LIB)
    STAMP.write_text(json.dumps({"sources_sha256": source_digest(), "arch": ARCH,
                                 "flags": _portable_flags(), "hipcc": hipcc}))
    if verbose:
        print(f"[spff] built {LIB.relative_to(ROOT)}")
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
