"""Shared pytest setup.

Markers:
  gpu  -- needs an MI355X (run with `-m gpu` on the GPU box); everything else
          runs on a CPU-only container.
"""
import glob
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("audio-fir-filter_amd", "oracle"):
    p = os.path.join(ROOT, sub)
    if p not in sys.path:
        sys.path.insert(0, p)
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN_DIR = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: requires an MI355X GPU (gfx950)")
    config.addinivalue_line("markers", "slow: long-running case")


def golden_names():
    return sorted(os.path.splitext(os.path.basename(p))[0]
                  for p in glob.glob(os.path.join(GOLDEN_DIR, "*.npz")))


def load_golden(name):
    with np.load(os.path.join(GOLDEN_DIR, f"{name}.npz"), allow_pickle=False) as d:
        return {k: d[k] for k in d.files}


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.load()
    return oracle
