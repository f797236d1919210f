import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cuda-phdslam_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box via gpurun)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def built():
    """Build libphdslam.so, the drop-in driver, the shim harness (tests/test_gpu_shim.py)
    and the oracle in-tree (hipcc cross-compiles without a GPU); each output is
    written under a per-process name and renamed, so parallel workers never race."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("phd_build", os.path.join(REPO, "cuda-phdslam_amd", "build.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    mod.build_lib()
    mod.build_driver()
    mod.build_shim_harness()
    mod.build_oracle()
    return True


@pytest.fixture(scope="session")
def gpu(built):
    import phdslam
    if phdslam.device_count() < 1:
        pytest.fail("gpu-marked test but no HIP device is visible (the HIP path has no CPU fallback)")
    return 0
