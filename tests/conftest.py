import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import rsa_pkg  # noqa: E402

rsa_pkg.load()

GOLDEN = os.path.join(ROOT, 'tests', 'golden')


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (runs the HIP library)')


def golden_cases():
    return sorted(d for d in os.listdir(GOLDEN) if os.path.isdir(os.path.join(GOLDEN, d)))


@pytest.fixture(scope='session')
def engine():
    from ruleset_analysis_amd.engine import Engine
    eng = Engine(0)
    yield eng
    eng.close()
