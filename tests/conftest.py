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


# Heartbeat for long tests (the baseline-size parity tests spend minutes in the CPU
# oracle without output): every 60 s a line on the terminal and in
# gpurun_out/heartbeat.log, so a long but live test is not mistaken for a hung one.
import threading  # noqa: E402
import time  # noqa: E402

import pytest  # noqa: E402


@pytest.fixture(autouse=True)
def _heartbeat(request):
    tr = request.config.pluginmanager.getplugin("terminalreporter")
    stop = threading.Event()
    t0 = time.time()
    name = request.node.nodeid
    out = ROOT / "gpurun_out"

    def beat():
        while not stop.wait(60.0):
            msg = f"[heartbeat] {name} running {time.time() - t0:.0f} s"
            try:
                if tr is not None:
                    tr.write_line(msg)
                if out.is_dir():
                    with open(out / "heartbeat.log", "a") as f:
                        f.write(msg + "\n")
            except Exception:
                pass

    th = threading.Thread(target=beat, daemon=True)
    th.start()
    yield
    stop.set()


# Long tests last.  pytest collects files alphabetically, which put the minutes-long
# baseline-size parity tests first: a run cut off by a time limit then lost the cheap
# per-op / network / 3DUNet / Swin / train tests instead of the expensive ones.  Stable
# sort: every other test keeps its order.
_LONG = (
    ("test_gpu_sharded.py", "test_depth_sharded_world8_f16x3_overlapped"),
    ("test_gpu_volume512.py", None),
    ("test_gpu_baseline_sizes.py", None),
)


def _long_rank(item):
    fname = pathlib.Path(str(item.fspath)).name
    for i, (f, name) in enumerate(_LONG):
        if fname == f and (name is None or item.name.split("[")[0] == name):
            return i + 1
    return 0


def pytest_collection_modifyitems(session, config, items):
    items.sort(key=_long_rank)
