import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "rust-bitcoinconsensus_amd")
for p in (ROOT, PKG, os.path.dirname(os.path.abspath(__file__))):
    if p not in sys.path:
        sys.path.insert(0, p)


import pytest  # noqa: E402

# Every device round of the suite runs through the device path (the stub device on the CPU, the
# HIP kernels on the GPU), tiny ones included: the library's default sends rounds of <= 16 checks
# to its host lane code (bcc_set_host_small_round), which test_host_verify*.py cover on their own.
os.environ.setdefault("BCC_HOST_SMALL_ROUND", "0")


@pytest.fixture(autouse=True)
def _gpu_rounds_ran_on_the_gpu(request):
    """Every -m gpu test must exercise the HIP kernels: a device round that failed and was
    verified on the host CPU (the library's failure policy) fails the test."""
    if request.node.get_closest_marker("gpu") is None:
        yield
        return
    import bitcoinconsensus_amd as B
    before = B.host_fallback_rounds()
    yield
    assert B.host_fallback_rounds() == before, \
        "a device round failed and was verified on the host CPU (see stderr)"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
