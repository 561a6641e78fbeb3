"""THINGS concept path: concept-mean activations paired with
behavioural embeddings (visreps/analysis/alignment.py:117-162) and the exact re-extraction
average (visreps/analysis/rsa.py:284-305). Host logic, CPU."""
import numpy as np
import torch

from visreps_amd.analysis.alignment import prepare_concept_alignment
from visreps_amd.analysis.rsa import _concept_average_exact


def _things(seed=0):
    r = np.random.RandomState(seed)
    keys = [f"img{i:03d}" for i in range(30)]
    image_ids = {"zebra": ["img003", "img001", "missing_a"], "apple": ["img010"],
                 "ghost": ["missing_b"], "boat": ["img020", "img021", "img029", "img000"]}
    emb = {c: r.randn(5).astype(np.float64) for c in image_ids}
    acts = {"fc": torch.from_numpy(r.randn(30, 7).astype(np.float32)),
            "conv": torch.from_numpy(r.randn(30, 2, 3).astype(np.float32))}
    return keys, {"image_ids": image_ids, "embeddings": emb}, acts


def test_concept_alignment_order_means_and_filtering():
    keys, raw, acts = _things()
    data = prepare_concept_alignment({}, acts, raw, keys)
    assert data.stimulus_ids == ["zebra", "apple", "boat"]  # dict order, empty concept dropped
    assert data.concept_image_ids["zebra"] == ["img003", "img001"]
    k = {s: i for i, s in enumerate(keys)}
    for layer, a in acts.items():
        got = data.activations[layer]
        assert got.dtype == a.dtype and got.shape == (3,) + tuple(a.shape[1:])
        for ci, c in enumerate(data.stimulus_ids):
            rows = [k[s] for s in data.concept_image_ids[c]]
            assert torch.allclose(got[ci], a[rows].float().mean(0), atol=0, rtol=0)
    assert data.neural.dtype == torch.float32
    assert np.array_equal(data.neural.numpy(),
                          np.stack([raw["embeddings"][c] for c in data.stimulus_ids]).astype(np.float32))


def test_concept_average_exact_reorders_by_ids():
    keys, raw, acts = _things(1)
    data = prepare_concept_alignment({}, acts, raw, keys)
    perm = np.random.RandomState(2).permutation(30)
    raw_ids = [keys[i] for i in perm]
    got = _concept_average_exact(acts["fc"][perm], raw_ids, data)
    assert torch.equal(got, data.activations["fc"])
