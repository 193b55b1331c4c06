import glob
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (os.path.join(ROOT, "oracle"), os.path.join(ROOT, "3d-hashjoin_amd", "python"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libhj3d.so on the device)")
    # Build the C restatement (oracle) and the HIP library if they are missing: both are
    # in-tree, git-ignored build outputs.
    if not os.path.exists(os.path.join(ROOT, "oracle", "liboracle.so")):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "oracle"], check=True,
                       stdout=subprocess.DEVNULL)
    if not os.path.exists(os.path.join(ROOT, "3d-hashjoin_amd", "lib", "libhj3d.so")):
        subprocess.run(["make", "-C", os.path.join(ROOT, "3d-hashjoin_amd"), "-j8"], check=True,
                       stdout=subprocess.DEVNULL)


def is_headline(g) -> bool:
    """Fixtures at the BASELINE headline sizes (configs B / C: |S| = 1e8; config E: log2R = 22).
    The generic per-fixture parity tests skip them; tests/test_gpu_headline.py runs them."""
    return g.get("nS", 0) >= 100_000_000 or g.get("log2R", 0) >= 22


def load_golden(pattern="*.json", headline=True):
    out = []
    for f in sorted(glob.glob(os.path.join(GOLDEN, pattern))):
        with open(f) as fh:
            g = json.load(fh)
        if headline or not is_headline(g):
            out.append((os.path.basename(f)[:-5], g))
    return out


@pytest.fixture(scope="session")
def ctx():
    import hj3d
    c = hj3d.Context(0)
    yield c
    c.close()
