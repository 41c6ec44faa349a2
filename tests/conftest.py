"""Test configuration.

`-m "not gpu"` tests run on CPU (oracle vs golden fixtures, host logic, ABI
export checks); `-m gpu` tests are the parity tests proper and call the HIP
path through the C ABI on an MI355X.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "vision-language-pretraining-for-bone-tumor-detection_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")
