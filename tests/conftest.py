import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.lib()
    O.set_threads(min(16, len(os.sched_getaffinity(0))))
    return O


@pytest.fixture(scope="session")
def golden():
    import json
    import numpy as np
    gdir = os.path.join(ROOT, "tests", "golden")
    man = json.load(open(os.path.join(gdir, "manifest.json")))
    cases = {}
    for name, meta in man["cases"].items():
        with np.load(os.path.join(gdir, meta["file"]), allow_pickle=False) as z:
            arrs = {k: z[k] for k in z.files}
        cases[name] = dict(meta, **arrs)
    return cases
