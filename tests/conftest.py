"""pytest configuration: the `gpu` marker and import paths.

`-m "not gpu"` runs here (no GPU): the oracle against the golden vectors,
host logic, and the C-ABI library's exports.  `-m gpu` runs on an MI355X and
holds the parity tests proper (HIP path vs oracle / golden fixtures).
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("", "oracle", "ipm-zoo_amd"):
    p = os.path.join(REPO, sub)
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
