import os
import sys
import pathlib

ROOT = pathlib.Path(__file__).resolve().parents[1]
PKG = ROOT / "spff-unet-spcct_amd"
for p in (str(ROOT), str(PKG)):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running test")
