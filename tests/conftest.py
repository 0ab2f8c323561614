import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "turbopfor-cpp_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "variants: measurement tools outside the library (scripts/build_variants.sh); "
                                       "run with -m variants on a GPU box")


def pytest_collection_modifyitems(config, items):
    # GPU tests are skipped automatically when no HIP device is visible, so a
    # plain `pytest tests/` on a CPU box stays green; `-m gpu` on the GPU box
    # runs them for real (and they fail loudly if the HIP library is missing).
    try:
        import torch

        have_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        have_gpu = False
    if have_gpu:
        return
    skip = pytest.mark.skip(reason="no HIP device visible")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
