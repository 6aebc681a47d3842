"""Test configuration: the `gpu` marker, import paths, shared golden-fixture helpers.

`-m "not gpu"` runs everywhere (oracle vs golden vectors, host logic, C-ABI load/exports, gloo
multi-process exchange); `-m gpu` are the parity tests proper and need an MI355X.
"""

import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (os.path.join(REPO, "ad-federatedlearning_amd"), os.path.join(REPO, "oracle"),
          os.path.join(REPO, "tests"), os.path.join(REPO, "tests", "golden"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); parity tests through the C ABI")
