import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# The parity tests force kernel shapes and walks through the GWAMD_* tuning
# variables, which libgwamd.so reads only with GWAMD_DIAG=1 (a drop-in user's
# environment never changes which kernel runs).  Tests of that gating clear
# it themselves.
os.environ.setdefault("GWAMD_DIAG", "1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); parity tests through the C ABI")
    config.addinivalue_line("markers", "slow: longer CPU-side oracle runs")
