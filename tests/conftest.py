"""Shared pytest configuration: the `gpu` marker and repo-root imports.

`-m "not gpu"` runs here (no GPU): oracle vs reference fixtures, host logic, the native
library's exports and host-side RNG. `-m gpu` runs on an MI355X and checks the HIP path
against the oracle."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP (MI355X) device")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def dev():
    import torch

    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    # Several tests extract the same stimuli twice (the eval, then the oracle's
    # re-derivation) and compare at 1e-12. The fc layers' GEMMs are not bit-reproducible run
    # to run by default (atomic split-K; measured 4e-7 on fc1, scripts/debug_extract_det.py);
    # deterministic algorithms make every re-extraction bit-identical.
    torch.use_deterministic_algorithms(True, warn_only=True)
    torch.backends.cudnn.deterministic = True
    return torch.device("cuda", 0)


@pytest.fixture(autouse=True)
def _release_device_memory(request):
    """GPU tests at bench and cfg3 sizes hold tens of GB each (workspaces, plans, RDMs):
    after every GPU test drop the library's scratch pool and torch's cached blocks, so
    the next test starts from an empty device (the suite runs in one process)."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    import gc

    import torch

    if not torch.cuda.is_available():
        return
    from visreps_amd._lib import workspace

    workspace.release()
    gc.collect()
    torch.cuda.empty_cache()


def record_margin(test: str, **values) -> None:
    """Append one measured parity margin (|dSpearman|, RDM error ...) as a JSON line to
    gpurun_out/parity_margins.jsonl (VISREPS_MARGINS overrides the path): the numbers behind
    each tolerance, committed under profiles/ from a GPU run."""
    import json

    path = os.environ.get("VISREPS_MARGINS", os.path.join(ROOT, "gpurun_out", "parity_margins.jsonl"))
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "a") as f:
        f.write(json.dumps({"test": test, **{k: (float(v) if hasattr(v, "__float__") else v)
                                             for k, v in values.items()}}) + "\n")
