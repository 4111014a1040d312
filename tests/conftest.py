import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# the tests drive internal switches (pool sizes, route variants, ...) through
# nmg_options.flags; the library accepts bits outside NMG_F_ALL only with this
os.environ.setdefault("NMG_INTERNAL_FLAGS", "1")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")


def _ensure_built():
    # build products are git-ignored; build them once per session if missing
    if not os.path.exists(os.path.join(ROOT, "oracle", "liboracle.so")):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, stdout=subprocess.DEVNULL)
    if not os.path.exists(os.path.join(ROOT, "numamma_amd", "libnumamma_gpu.so")):
        subprocess.run(["make", "-C", os.path.join(ROOT, "numamma_amd")], check=True, stdout=subprocess.DEVNULL)


_ensure_built()


@pytest.fixture(scope="session")
def gpu_available():
    import torch

    return torch.cuda.is_available()


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.device_count() > 0:
        return
    skip = pytest.mark.skip(reason="no GPU visible")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
