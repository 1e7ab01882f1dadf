import json
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running")
    lib = ROOT / "oracle" / "build" / "libhbec_oracle.so"
    if not lib.exists():
        subprocess.run(["make", "-C", str(ROOT / "oracle")], check=True, capture_output=True)


@pytest.fixture(scope="session")
def kats():
    return json.loads((GOLDEN / "kats.json").read_text())


@pytest.fixture(scope="session")
def vectors():
    return json.loads((GOLDEN / "vectors.json").read_text())
