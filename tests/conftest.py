"""pytest setup: `gpu` marker, repo on sys.path, in-tree builds present."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")


def _ensure_built():
    # Libraries are git-ignored build outputs; build them if this checkout has none.
    if not os.path.exists(os.path.join(ROOT, "oracle", "build", "liboracle.so")) or \
            not os.path.exists(os.path.join(ROOT, "oracle", "build", "ref_tests")):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    if not os.path.exists(os.path.join(ROOT, "ggrs_amd", "libggrs_amd.so")):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "ggrs_amd", "csrc")], check=True)


_ensure_built()


@pytest.fixture(scope="session")
def gpu_available():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    return True
