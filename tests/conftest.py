import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, 'ctpa-clip_amd')
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, 'tests', 'golden')


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (run via gpurun)')
    config.addinivalue_line('markers', 'slow: multi-second CPU oracle runs at base config')


@pytest.fixture(scope='session')
def golden_tiny():
    from safetensors.torch import load_file
    return load_file(os.path.join(GOLDEN, 'golden_tiny.safetensors'))


@pytest.fixture(scope='session')
def golden_base():
    from safetensors.torch import load_file
    path = os.path.join(GOLDEN, 'golden_base_b2.safetensors')
    if not os.path.exists(path):
        pytest.skip('base fixture not generated')
    return load_file(path)
