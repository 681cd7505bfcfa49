import importlib
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs under gpurun)")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as o
    o.build()
    return o


@pytest.fixture(scope="session")
def fec():
    """The product package (0xfec_amd) — its directory name starts with a digit, so it is
    imported by name."""
    return importlib.import_module("0xfec_amd")


@pytest.fixture
def tune(fec):
    """tune(knob=value, ...): set process-wide kernel-selection knobs (Codec.set_tuning) for one
    test; every knob set is restored afterwards."""
    codec, saved = [], {}

    def set_knobs(**kv):
        if not codec:
            codec.append(fec.Codec(0))
        old = codec[0].set_tuning(**kv)
        for k_, v in old.items():
            saved.setdefault(k_, v)

    yield set_knobs
    if codec:
        codec[0].set_tuning(**saved)
        codec[0].close()


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "reference_cases.json")) as f:
        return json.load(f)
