import os
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")
    config.addinivalue_line("markers", "gpu_slow: a GPU stress matrix, run with KUNGFU_AMD_GPU_SLOW=1")


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle
    oracle.build()
    return oracle


# Stress matrices (many strategy x piece x stage combinations of one path)
# carry `gpu_slow` besides `gpu`: `-m gpu` skips them unless
# KUNGFU_AMD_GPU_SLOW=1, so the driver's suite keeps one oracle-checked case
# of every path inside its time limit; the builder runs the whole matrix with
# KUNGFU_AMD_GPU_SLOW=1 (profiles/rNN/pytest_gpu_slow_*.txt).
def pytest_collection_modifyitems(config, items):
    if os.environ.get("KUNGFU_AMD_GPU_SLOW") == "1":
        return
    skip = pytest.mark.skip(reason="gpu_slow: set KUNGFU_AMD_GPU_SLOW=1 to run")
    for it in items:
        if "gpu_slow" in it.keywords:
            it.add_marker(skip)
