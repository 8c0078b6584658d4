#!/usr/bin/env python3
"""Build a variant of libspff_hip.so with extra compile flags (kernel tuning
experiments), e.g.

    python scripts/build_variant.py variants/libspff_iglp0.so -DSPFF_XIGLP=0

Select it at run time with SPFF_LIB=<path> (innovative3D._engine.lib_path)."""
import concurrent.futures as cf
import pathlib
import subprocess
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "spff-unet-spcct_amd"))
import build_ext as B  # noqa: E402

out = pathlib.Path(sys.argv[1]).resolve()
extra = sys.argv[2:]
obj = ROOT / "spff-unet-spcct_amd" / "build" / ("obj_" + out.stem)
obj.mkdir(parents=True, exist_ok=True)
out.parent.mkdir(parents=True, exist_ok=True)
hipcc = B._hipcc()


def one(src):
    o = obj / (src.stem + ".o")
    r = subprocess.run([hipcc, *B.FLAGS, *extra, "-c", str(src), "-o", str(o)], capture_output=True,
                       text=True)
    if r.returncode:
        raise SystemExit(f"{src.name}: {r.stderr[-3000:]}")
    return o


with cf.ThreadPoolExecutor(8) as ex:
    objs = list(ex.map(one, B.sources()))
r = subprocess.run([hipcc, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", str(out),
                    *map(str, objs)], capture_output=True, text=True)
if r.returncode:
    raise SystemExit(r.stderr[-3000:])
print(f"built {out}")
