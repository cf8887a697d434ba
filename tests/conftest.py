import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from simclr_pytorch_distributed_amd.ops import _ext
    m = _ext.require()  # native path must load on a GPU box (fail loudly, never fall back)
    var = os.environ.get("SDX_EXT_VARIANT", "")
    assert not var or m.__name__.endswith("_C_" + var), (m.__name__, var)   # e.g. the sanitizer build
    yield torch.device("cuda:0")
    # drop tensors kept alive for side-stream wgrads by tests that ran a backward
    # without an optimizer step / reducer join (ops/streams.py)
    from simclr_pytorch_distributed_amd.ops import streams
    torch.cuda.synchronize()
    streams.release()
