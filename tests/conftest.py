import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running")


# One parity test per BASELINE.json config (and per default kernel of the headline path) runs
# first, so that a `pytest -x` run that stops early has still exercised every config against
# the oracle or the golden fixtures.  (file, test name, substring of the parameter id or "")
PRIORITY = [
    ("test_gpu_parity.py", "test_three_pass_vs_oracle", ""),          # 256^3 default: k_tp_mid_sw + LDS-DMA
    ("test_gpu_parity.py", "test_three_pass_100_vs_oracle", ""),      # 100^3 default mesh: radix-10 3-sweep (AUTO)
    ("test_gpu_parity.py", "test_plane_vs_oracle", "100x100x100"),    # 100^3 plane schedule (selectable)
    ("test_gpu_parity.py", "test_plane_vs_oracle", "64x64x64"),
    ("test_gpu_parity.py", "test_vs_oracle", "128x128x128"),          # config 2
    ("test_transport.py", "test_driver_fft_pc_matches_oracle", ""),   # config 1 (32^3 GMRES + PCSHELL)
    ("test_transport.py", "test_config3_256_converges_and_solves", ""),  # config 3
    ("test_wave.py", "test_wave_plan_128_inverts_periodic_operator", ""),  # config 4
    ("test_wave.py", "test_wave_plan_128_three_sweep_matches_oracle", ""),  # config 4, 3 sweeps
    ("test_dist_gpu.py", "test_group_config5_512_in_8_slabs", ""),    # config 5 (HIP path, 8 slabs)
    ("test_dist_gpu.py", "test_slab_plan_processes_vs_oracle", ""),   # config 5 pieces, several processes
    ("test_pcshell_mpi_gpu.py", "", ""),                              # PCSHELL on a 2-rank communicator
]


def _priority(item):
    fname = os.path.basename(str(item.fspath))
    name = item.originalname or item.name
    for k, (f, t, p) in enumerate(PRIORITY):
        if fname == f and (not t or name == t) and p in item.name:
            return k
    return len(PRIORITY)


def pytest_collection_modifyitems(session, config, items):
    # stable: everything else keeps its collection order behind the priority tests
    items[:] = sorted(items, key=_priority)


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
