"""pytest configuration: the `gpu` marker and shared paths.

`-m "not gpu"` (this container, no GPU): oracle vs golden fixtures, host
logic (event loop, streams, stage error paths, sharding over gloo) and the
C-ABI library's exported symbols.  `-m gpu` (MI355X box): HIP kernels and
stages, through the C ABI, against the oracle and the fixtures.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running (seconds to a minute)")
