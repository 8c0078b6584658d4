#!/usr/bin/env python3
"""Build libspff_hip.so from the csrc/ and include/ of a git revision (default HEAD) into
an output path, for A/B runs against the working tree (SPFF_LIB=<out>):

    python scripts/build_rev.py abvar/libspff_head.so [REV] [extra hipcc flags]"""
import concurrent.futures as cf
import pathlib
import subprocess
import sys
import tempfile

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "spff-unet-spcct_amd"))
import build_ext as B  # noqa: E402

out = pathlib.Path(sys.argv[1]).resolve()
rev = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("-") else "HEAD"
extra = [a for a in sys.argv[2:] if a.startswith("-")]
tmp = pathlib.Path(tempfile.mkdtemp(prefix="spff_rev_"))
for sub in ("spff-unet-spcct_amd/csrc", "include"):
    files = subprocess.run(["git", "-C", str(ROOT), "ls-tree", "--name-only", rev, sub + "/"],
                           capture_output=True, text=True, check=True).stdout.split()
    (tmp / sub).mkdir(parents=True, exist_ok=True)
    for f in files:
        data = subprocess.run(["git", "-C", str(ROOT), "show", f"{rev}:{f}"], capture_output=True,
                              check=True).stdout
        (tmp / f).write_bytes(data)
csrc, inc = tmp / "spff-unet-spcct_amd/csrc", tmp / "include"
flags = [f for f in B.FLAGS if not f.startswith("-I")] + [f"-I{inc}", f"-I{csrc}"] + extra
hipcc = B._hipcc()


def one(src):
    o = src.with_suffix(".o")
    r = subprocess.run([hipcc, *flags, "-c", str(src), "-o", str(o)], capture_output=True, text=True)
    if r.returncode:
        raise SystemExit(f"{src.name}: {r.stderr[-3000:]}")
    return o


with cf.ThreadPoolExecutor(8) as ex:
    objs = list(ex.map(one, sorted(csrc.glob("*.hip"))))
out.parent.mkdir(parents=True, exist_ok=True)
r = subprocess.run([hipcc, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o", str(out),
                    *map(str, objs)], capture_output=True, text=True)
if r.returncode:
    raise SystemExit(r.stderr[-3000:])
print(f"built {out} from {rev}")
