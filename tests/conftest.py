"""Test configuration.

* ``gpu`` marks tests that need an MI355X (run with ``-m gpu`` on the GPU box);
  everything else runs on the CPU-only build container.
* The repo root (for ``oracle``) and ``muzero-go_amd`` (for the ``mzgo``
  package) go on ``sys.path``.
"""
import os
import sys

import pytest
import torch

# The golden vectors were recorded with one intra-op thread; oneDNN's conv
# reduction order (hence the last ulp) depends on the thread count.
torch.set_num_threads(1)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "muzero-go_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU (HIP engine)")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN
