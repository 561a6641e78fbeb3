"""The import surface of the reference's own test modules, on this package.

A user who points the reference's tests at visreps_amd needs every name they import to
exist with the reference's call shape. The lists below are the imports of
/root/reference/tests/test_rsa_bootstrap.py (lines 42-54, 696, 1505, 1943) and
/root/reference/tests/test_encoding_score.py (lines 47-56), plus the module attributes those
tests touch (`visreps.utils._RESULTS_DB_PATH`, `visreps.evals.eval`). CPU only: nothing here
calls the HIP library.
"""
import inspect

import pytest

REFERENCE_IMPORTS = {
    "visreps_amd.analysis.rsa": ["compute_rdm", "compute_rdm_correlation", "compute_rsa", "_kendall_tau_a",
                                 "_concept_average_exact", "_rank"],
    "visreps_amd.analysis.alignment": ["AlignmentData", "_align_stimulus_level", "prepare_concept_alignment",
                                       "prepare_traintest_alignment", "compute_traintest_alignment"],
    "visreps_amd.analysis.encoding_score": ["_znorm", "_znorm_fit", "_flatten_to_cpu", "_fit_and_score",
                                            "compute_encoding_score"],
    "visreps_amd.utils": ["save_results", "_compute_run_id", "_RESULTS_DB_PATH"],
    "visreps_amd.evals": ["eval"],
}


@pytest.mark.parametrize("module", sorted(REFERENCE_IMPORTS))
def test_reference_test_imports_resolve(module):
    import importlib

    mod = importlib.import_module(module)
    missing = [n for n in REFERENCE_IMPORTS[module] if not hasattr(mod, n)]
    assert not missing, f"{module} lacks {missing}"


def test_call_shapes_match_the_reference():
    # positional arities the reference's tests use
    from visreps_amd.analysis import encoding_score as E
    from visreps_amd.analysis import rsa as R

    assert list(inspect.signature(R._kendall_tau_a).parameters) == ["x", "y"]
    ps = inspect.signature(E._fit_and_score).parameters
    assert len(ps) == 6 and list(ps)[-1] == "backend"  # (X_tr, Y_tr, X_te, Y_te, alphas, backend)
    assert list(inspect.signature(E._flatten_to_cpu).parameters) == ["acts"]


def test_flatten_to_cpu_is_the_reference_helper():
    # /root/reference/tests/test_encoding_score.py:309-350: 4-D flattened, 2-D kept, CPU
    # float32 out, the input dict untouched
    import torch

    from visreps_amd.analysis.encoding_score import _flatten_to_cpu

    acts = {"conv": torch.randn(3, 2, 4, 4, dtype=torch.float64), "fc": torch.randn(3, 7)}
    out = _flatten_to_cpu(acts)
    assert out["conv"].shape == (3, 32) and out["fc"].shape == (3, 7)
    assert all(v.dtype == torch.float32 and v.device.type == "cpu" for v in out.values())
    assert acts["conv"].shape == (3, 2, 4, 4) and acts["conv"].dtype == torch.float64
    assert torch.equal(out["conv"], acts["conv"].reshape(3, -1).float())


def test_kendall_tau_a_short_input_needs_no_device():
    # rsa.py:25-26: n < 2 returns (nan, nan) before any arithmetic
    import math

    import numpy as np

    from visreps_amd.analysis.rsa import _kendall_tau_a

    t, p = _kendall_tau_a(np.array([1.0]), np.array([1.0]))
    assert math.isnan(t) and math.isnan(p)
