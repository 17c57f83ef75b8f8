import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "skyvault-rs_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running (GiB-scale) test")


@pytest.fixture(scope="session")
def oracle():
    import pyoracle

    pyoracle.build()
    return pyoracle


@pytest.fixture(autouse=True)
def _clear_test_hooks():
    """the library's test hooks (skv_test_option) are process-wide: none outlives its test"""
    yield
    api = sys.modules.get("skv.api")
    if api is not None and getattr(api, "_lib", None) is not None:
        api.test_option(None)
