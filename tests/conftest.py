import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

REF_DIR = os.path.join(ROOT, "oracle", "_ref")
REF_TOOL = os.path.join(REF_DIR, "ref_tool")
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")


@pytest.fixture(scope="session")
def ref_tool():
    """The reference codec compiled from /root/reference by oracle/Makefile
    (prebuilt here, travels to the GPU box).  Test infrastructure only."""
    if not os.path.exists(REF_TOOL):
        pytest.fail("oracle/_ref/ref_tool missing: run __graft_entry__.build() "
                    "in the container that has /root/reference")
    return REF_TOOL


def run_ref(*args, jobs=8):
    cmd = [REF_TOOL, "jobs", str(jobs)] + [str(a) for a in args]
    subprocess.run(cmd, check=True)


@pytest.fixture(scope="session")
def engine_lib():
    from pairphone_amd import load_library
    return load_library()


@pytest.fixture(autouse=True)
def _torch_hip_first(request):
    """GPU tests: bring up torch's HIP context before the engine library
    makes its first HIP call, so tests that mix the C ABI with torch device
    buffers see the same device set in any order."""
    gpu = request.node.get_closest_marker("gpu") is not None
    if gpu:
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    yield
    if gpu:
        # hand the device memory this test's tensors held back to the device:
        # the suite runs in one process, and later tests start other
        # processes on the same GPU (tests/test_shard.py), whose kernels need
        # their own scratch
        import gc
        import torch
        gc.collect()
        if torch.cuda.is_available():
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
