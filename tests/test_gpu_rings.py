"""Host rings under more callers than rings.

A fresh child process (tests/ring_stress.py) runs with HBEC_HOST_RINGS=2:
16 threads of hbec_encode_host / hbec_encode_host_md5 / hbec_reconstruct_host
on pageable and pinned stripes, every result compared with the oracle.  It
must finish inside DEADLINE_S; round 2's soak once made no progress for
300 s while callers created rings on demand."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]
# the child computes the oracle for 16 threads on the box's CPU share: 20-40 s
# on most boxes, 90+ on one slow box in round 6 (its whole suite ran 3x slower)
DEADLINE_S = 150


@pytest.mark.timeout(170)
def test_more_callers_than_rings_finish_and_match_oracle():
    env = dict(os.environ, HBEC_HOST_RINGS="2")
    p = subprocess.run([sys.executable, str(ROOT / "tests" / "ring_stress.py"), "16", "6"], env=env,
                       capture_output=True, text=True, timeout=DEADLINE_S)
    assert p.returncode == 0, p.stdout + p.stderr
    res = json.loads(p.stdout.strip().splitlines()[-1])
    assert res["calls"] == 16 * 6 and not res["errors"], res
