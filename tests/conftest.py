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
    _start_heartbeat()


def _start_heartbeat():
    """On the GPU box (GRAFT_REPO_ROOT set): append the running test's id to
    gpurun_out/heartbeat.txt every 30 s, so a long oracle sweep (pytest writes
    its log only between tests) is not taken for a hung run."""
    root = os.environ.get("GRAFT_REPO_ROOT")
    if not root:
        return
    import threading
    import time
    path = os.path.join(root, "gpurun_out", "heartbeat.txt")

    def beat():
        while True:
            time.sleep(30)
            try:
                os.makedirs(os.path.dirname(path), exist_ok=True)
                with open(path, "a") as fh:
                    fh.write(f"{time.strftime('%H:%M:%S')} {os.environ.get('PYTEST_CURRENT_TEST', '-')}\n")
            except OSError:
                pass

    threading.Thread(target=beat, daemon=True).start()


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
