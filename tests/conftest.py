"""Test configuration: the `gpu` marker and import paths.

`-m "not gpu"` runs on any host (oracle vs golden vectors, host logic, ABI exports);
`-m gpu` needs an MI355X and exercises the HIP path through the C ABI.
"""
import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT, ROOT / "api-ratelimit_amd", ROOT / "oracle"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD MI355X GPU (runs the HIP path)")


@pytest.fixture(scope="session")
def golden():
    import json
    return json.loads((ROOT / "tests" / "golden" / "reference_vectors.json").read_text())
