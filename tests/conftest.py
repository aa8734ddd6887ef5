import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))
# No HSA_ENABLE_IPC_MODE_LEGACY here: libishmem_amd sets it when it loads (runtime.cpp
# ipc_mode_default), and the multi-process tests remove it from their PEs' environments.


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running")
