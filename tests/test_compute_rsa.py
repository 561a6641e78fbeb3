"""compute_rsa behaviour (reference: visreps/analysis/rsa.py:132-281), transcribed from the
reference's own tests (tests/test_rsa_bootstrap.py:567-584 re_extract_fn, :606-622 no
input mutation, :645 n_select=None, :1439 re_extract_fn changes the test RDM, :2058
n_bootstrap=1, :2100 4-D conv activations, plus reproducibility / seeds / defaults)
against the HIP path, with the values pinned to the CPU oracle where they have one."""
import numpy as np
import pytest
import torch

from oracle import rsa_oracle as O

pytestmark = pytest.mark.gpu


def _data(seed=42, n_train=200, n_test=50, v=100, noise=0.5, shape=None):
    rng = np.random.RandomState(seed)
    nt = rng.randn(n_train, v).astype(np.float32)
    ne = rng.randn(n_test, v).astype(np.float32)
    good = (nt + noise * rng.randn(n_train, v)).astype(np.float32), (ne + noise * rng.randn(n_test, v)).astype(np.float32)
    bad = rng.randn(n_train, v).astype(np.float32), rng.randn(n_test, v).astype(np.float32)
    if shape is not None:
        good = tuple(g.reshape((-1,) + shape) for g in good)
        bad = tuple(b.reshape((-1,) + shape) for b in bad)
    return {"good": good, "bad": bad}, nt, ne


def _split(layers, nt, ne, dev):
    from visreps_amd.analysis.alignment import AlignmentData

    ids = [str(i) for i in range(ne.shape[0])]
    tr = AlignmentData({k: torch.from_numpy(v[0]).to(dev) for k, v in layers.items()}, torch.from_numpy(nt).to(dev))
    te = AlignmentData({k: torch.from_numpy(v[1]).to(dev) for k, v in layers.items()}, torch.from_numpy(ne).to(dev),
                       stimulus_ids=ids)
    return tr, te


def _oracle(layers, nt, ne, **kw):
    return O.compute_rsa({"compare_method": kw.pop("method", "spearman")},
                         {k: v[0] for k, v in layers.items()}, nt,
                         {k: v[1] for k, v in layers.items()}, ne, **kw)[0]


def _close(got, ref, tol=1e-5):
    assert got["layer"] == ref["layer"]
    assert abs(got["score"] - ref["score"]) < tol
    for g, r in zip(got["layer_selection_scores"], ref["layer_selection_scores"]):
        assert g["layer"] == r["layer"] and abs(g["score"] - r["score"]) < tol
    if ref.get("bootstrap_scores") is not None:
        assert np.max(np.abs(np.asarray(got["bootstrap_scores"]) - ref["bootstrap_scores"])) < tol


def test_re_extract_fn_called_once_with_best_layer(dev):
    from visreps_amd.analysis.rsa import compute_rsa

    layers, nt, ne = _data()
    tr, te = _split(layers, nt, ne, dev)
    calls = []

    def re_extract(layer, stimulus_ids=None):
        calls.append((layer, stimulus_ids))
        return te.activations[layer], te.stimulus_ids

    got = compute_rsa({"compare_method": "spearman"}, tr, te, n_select=100, bootstrap=False, seed=42,
                      re_extract_fn=re_extract)[0]
    assert calls == [("good", te.stimulus_ids)]
    _close(got, _oracle(layers, nt, ne, n_select=100, bootstrap=False, seed=42))


def test_re_extract_fn_output_is_the_test_rdm(dev):
    # the re-extracted activations, not the split's own, build the test model RDM
    from visreps_amd.analysis.rsa import compute_rsa

    layers, nt, ne = _data()
    tr, te = _split(layers, nt, ne, dev)
    exact = np.random.RandomState(7).randn(*layers["good"][1].shape).astype(np.float32) + layers["good"][1]
    got = compute_rsa({"compare_method": "spearman"}, tr, te, n_select=100, bootstrap=True, n_bootstrap=25,
                      seed=42, re_extract_fn=lambda l, s=None: (torch.from_numpy(exact).to(dev), s))[0]
    plain = compute_rsa({"compare_method": "spearman"}, tr, te, n_select=100, bootstrap=True, n_bootstrap=25,
                        seed=42)[0]
    assert got["score"] != plain["score"]
    swapped = {"good": (layers["good"][0], exact), "bad": layers["bad"]}
    _close(got, _oracle(swapped, nt, ne, n_select=100, bootstrap=True, n_bootstrap=25, seed=42))


def test_does_not_mutate_inputs(dev):
    from visreps_amd.analysis.rsa import compute_rsa

    layers, nt, ne = _data()
    tr, te = _split(layers, nt, ne, dev)
    before = ([t.clone() for t in tr.activations.values()], [t.clone() for t in te.activations.values()],
              tr.neural.clone(), te.neural.clone())
    compute_rsa({"compare_method": "spearman"}, tr, te, n_select=100, bootstrap=True, n_bootstrap=10, seed=42)
    for a, b in zip(before[0], tr.activations.values()):
        assert torch.equal(a, b)
    for a, b in zip(before[1], te.activations.values()):
        assert torch.equal(a, b)
    assert torch.equal(before[2], tr.neural) and torch.equal(before[3], te.neural)


def test_n_select_none_uses_all_train(dev):
    from visreps_amd.analysis.rsa import compute_rsa

    layers, nt, ne = _data()
    tr, te = _split(layers, nt, ne, dev)
    got = compute_rsa({"compare_method": "spearman"}, tr, te, n_select=None, bootstrap=True, n_bootstrap=20,
                      seed=42)[0]
    _close(got, _oracle(layers, nt, ne, n_select=None, bootstrap=True, n_bootstrap=20, seed=42))
    # n_select >= n_train also means all rows and draws nothing from the stream
    again = compute_rsa({"compare_method": "spearman"}, tr, te, n_select=500, bootstrap=True, n_bootstrap=20,
                        seed=42)[0]
    assert again["bootstrap_scores"] == got["bootstrap_scores"]


def test_n_bootstrap_1(dev):
    from visreps_amd.analysis.rsa import compute_rsa

    layers, nt, ne = _data()
    tr, te = _split(layers, nt, ne, dev)
    got = compute_rsa({"compare_method": "spearman"}, tr, te, n_select=50, bootstrap=True, n_bootstrap=1,
                      seed=42)[0]
    assert len(got["bootstrap_scores"]) == 1
    assert got["ci_low"] == got["ci_high"] == got["bootstrap_scores"][0]
    _close(got, _oracle(layers, nt, ne, n_select=50, bootstrap=True, n_bootstrap=1, seed=42))


def test_4d_conv_activations_are_flattened(dev):
    from visreps_amd.analysis.rsa import compute_rsa

    layers, nt, ne = _data(v=64 * 3 * 3, shape=(64, 3, 3))
    tr, te = _split(layers, nt.reshape(nt.shape[0], -1), ne.reshape(ne.shape[0], -1), dev)
    got = compute_rsa({"compare_method": "spearman"}, tr, te, n_select=30, bootstrap=True, n_bootstrap=10,
                      seed=42)[0]
    flat = {k: (v[0].reshape(v[0].shape[0], -1), v[1].reshape(v[1].shape[0], -1)) for k, v in layers.items()}
    _close(got, _oracle(flat, nt, ne, n_select=30, bootstrap=True, n_bootstrap=10, seed=42))


def test_reproducible_and_seed_dependent(dev):
    from visreps_amd.analysis.rsa import compute_rsa

    layers, nt, ne = _data()
    tr, te = _split(layers, nt, ne, dev)
    r1 = compute_rsa({"compare_method": "spearman"}, tr, te, n_select=100, n_bootstrap=20, seed=42)[0]
    r2 = compute_rsa({"compare_method": "spearman"}, tr, te, n_select=100, n_bootstrap=20, seed=42)[0]
    r3 = compute_rsa({"compare_method": "spearman"}, tr, te, n_select=100, n_bootstrap=20, seed=99)[0]
    assert r1["score"] == r2["score"] and r1["ci_low"] == r2["ci_low"] and r1["ci_high"] == r2["ci_high"]
    assert r1["bootstrap_scores"] == r2["bootstrap_scores"]
    assert r1["bootstrap_scores"] != r3["bootstrap_scores"]


def test_defaults_and_kendall(dev):
    from visreps_amd.analysis.rsa import compute_rsa

    layers, nt, ne = _data()
    tr, te = _split(layers, nt, ne, dev)
    got = compute_rsa({}, tr, te, n_select=100, bootstrap=False, seed=42)[0]
    assert got["compare_method"] == "spearman" and got["analysis"] == "rsa"
    assert got["ci_low"] is None and "bootstrap_scores" not in got
    kt = compute_rsa({"compare_method": "kendall"}, tr, te, n_select=100, bootstrap=True, n_bootstrap=15,
                     seed=42)[0]
    _close(kt, _oracle(layers, nt, ne, n_select=100, bootstrap=True, n_bootstrap=15, seed=42, method="kendall"))
