import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device")


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(ROOT, "tests", "golden")


@pytest.fixture
def knob_ctx(monkeypatch):
    """A factory of fresh contexts, each created with the given environment switches set: the
    library reads its switches (RC_DEC_PAIR, RC_STREAM_*, RC_PRIO, RC_HIST_HOT) once per
    context, in rc_ctx_create (include/range_coder.h), so a test that changes one needs a new
    context.  The contexts are closed after the test."""
    made = []

    def make(**env):
        import range_coder_rust_amd as rc
        for k, v in env.items():
            monkeypatch.setenv(k, str(v))
        c = rc.Context(0)
        made.append(c)
        return c

    yield make
    if made:
        import torch
        torch.cuda.synchronize()
    for c in made:
        c.close()
