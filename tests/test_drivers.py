"""The THINGS-behaviour and NSD-Synthetic eval drivers (reference: visreps/evals.py:95-155,
:404-548) and reconstruct_from_pcs inside the RSA phase 2 (:312-323), end to end on the
seeded synthetic stand-ins, re-derived with the CPU oracle from the same exact
activations.

Tolerances: the oracle is run on the product's own RDMs (rdm_fn = the HIP Gram), so
layer choice, selection scores, point estimate and bootstrap must agree to 1e-12; the
RDM kernel itself is checked against numpy's RDMs entry-wise (1e-5)."""
import numpy as np
import pytest
import torch

from oracle import pca_oracle as P
from oracle import rsa_oracle as O
from visreps_amd import utils
from conftest import record_margin

# |dSpearman| between the product and the all-oracle path at these small n (each side builds
# its own RDMs): the north-star bound, with the measured values logged by record_margin
TOL_SMALL_N = 1e-5

pytestmark = pytest.mark.gpu


def _cfg(items):
    cfg = utils.load_config("configs/eval/base.json", items + ["mode=eval"])
    return utils.validate_config(cfg)


def _model(cfg, dev):
    from visreps_amd import evals
    from visreps_amd.models import utils as mutils

    cfg = evals._load_cfg(cfg)
    return mutils.configure_feature_extractor(cfg, mutils.load_model(cfg, dev))


def _gpu_rdm(dev):
    from visreps_amd.analysis import rsa as R

    def fn(x):
        x = np.asarray(x, np.float32)
        g = R.compute_rdm(torch.from_numpy(x.reshape(x.shape[0], -1)).to(dev)).cpu().numpy()
        assert np.max(np.abs(g - O.compute_rdm(x.reshape(x.shape[0], -1)))) < 1e-5
        return g
    return fn


def _exact(model, stimuli, dev, layer, ids=None):
    from visreps_amd.dataloaders.neural import _make_loader
    from visreps_amd.models import utils as mutils

    acts, got = mutils.extract_single_layer(model, _make_loader(stimuli, None, 64, 0), dev, layer, ids)
    return acts.numpy(), got


# --------------------------------------------------------------------------- THINGS
def _things_vs_oracle(dev, n_concepts, n_images, n_boot):
    from visreps_amd import evals
    from visreps_amd.analysis.alignment import AlignmentData, prepare_concept_alignment
    from visreps_amd.analysis.rsa import _concept_average_exact
    from visreps_amd.dataloaders.neural import _make_loader, load_things_synthetic
    from visreps_amd.models import utils as mutils

    items = ["neural_dataset=things-behavior", f"synthetic.things_concepts={n_concepts}",
             f"synthetic.things_images={n_images}", f"n_bootstrap={n_boot}", "batchsize=128"]
    df = evals.eval(_cfg(items))
    assert len(df) == 1
    row = df.iloc[0]
    assert row["analysis"] == "rsa" and len(row["layer_selection_scores"]) == 14
    assert len(row["bootstrap_scores"]) == n_boot and row["ci_low"] <= row["ci_high"]

    # oracle: the same SRP concept means for selection, exact concept means for evaluation
    cfg = _cfg(items)
    model = _model(cfg, dev)
    targets, stimuli = load_things_synthetic(cfg)
    assert len(stimuli) == n_concepts * n_images
    acts, ids = mutils.get_activations(model, _make_loader(stimuli, None, 128, 0), dev,
                                       keep_on_device=True, srp_seed=cfg.srp_seed)
    conc = prepare_concept_alignment(cfg, acts, targets, ids)
    del acts
    perm = np.random.RandomState(42).permutation(n_concepts)
    n_sel = int(n_concepts * 0.2)  # evals.py:111-115
    sel, ev = perm[:n_sel], perm[n_sel:]
    concepts = conc.stimulus_ids
    sel_acts = {l: a.cpu().numpy()[sel] for l, a in conc.activations.items()}
    neural = conc.neural.numpy()
    evaluation = AlignmentData({}, conc.neural[ev], stimulus_ids=[concepts[i] for i in ev],
                               concept_image_ids={concepts[i]: targets["image_ids"][concepts[i]] for i in ev})

    class ExactMeans(dict):  # the oracle asks only for its best layer
        def __missing__(self, layer):
            # concept means of the exact activations on the device, as the eval forms them
            # (their arithmetic: tests/test_concepts.py)
            raw, raw_ids = mutils.extract_single_layer(model, _make_loader(stimuli, None, 128, 0), dev, layer,
                                                       keep_on_device=True)
            out = _concept_average_exact(raw, raw_ids, evaluation).cpu().numpy()
            del raw
            self[layer] = out
            return out

    ref = O.compute_rsa({"compare_method": "spearman"}, sel_acts, neural[sel], ExactMeans(),
                        neural[ev], n_select=None, bootstrap=True, n_bootstrap=n_boot, seed=42,
                        rdm_fn=_gpu_rdm(dev))[0]
    assert row["layer"] == ref["layer"]
    for g, r in zip(row["layer_selection_scores"], ref["layer_selection_scores"]):
        assert g["layer"] == r["layer"] and abs(g["score"] - r["score"]) <= 1e-12
    assert abs(row["score"] - ref["score"]) <= 1e-12
    assert np.max(np.abs(np.asarray(row["bootstrap_scores"]) - ref["bootstrap_scores"])) <= 1e-12
    return row


def test_things_behavior_end_to_end_matches_oracle(dev):
    _things_vs_oracle(dev, 60, 2, 15)


def test_things_behavior_full_size_matches_oracle(dev):
    """BASELINE configs[3] at its stated size: THINGS' 1,854 concepts x 14 images (25,956
    images, reference evals.py:95-155 / neural.py:313-335), 371 selection and 1,483
    evaluation concepts, through evals.eval and re-derived by the oracle on the product's
    RDMs (the RDM kernel itself vs numpy entry-wise, 1e-5, inside _gpu_rdm)."""
    row = _things_vs_oracle(dev, 1854, 14, 20)
    record_margin("things_full_size", concepts=1854, images=25956, score=row["score"])


def test_things_behavior_encoding_refused(dev):
    from visreps_amd import evals

    with pytest.raises((AssertionError, ValueError)):
        evals.eval(_cfg(["neural_dataset=things-behavior", "analysis=encoding_score",
                         "synthetic.things_concepts=20"]))


# --------------------------------------------------------------------------- NSD Synthetic
NSD_ITEMS = ["synthetic.n_test=80", "synthetic.n_train=120", "n_select=60", "n_bootstrap=12",
             "region=[V1,hV4]", "subject_idx=[0,1]", "batchsize=64", "synthetic.nsd_synthetic_n=70"]


def test_nsd_synthetic_reuses_nsd_layers_and_matches_oracle(dev, tmp_path, monkeypatch):
    from visreps_amd import evals
    from visreps_amd.dataloaders.neural import load_nsd_synthetic_test_data

    monkeypatch.setattr(utils, "_RESULTS_DB_PATH", tmp_path / "results.db")
    with pytest.raises(ValueError, match="Run NSD eval first"):
        evals.eval(_cfg(NSD_ITEMS + ["neural_dataset=nsd_synthetic"]))

    nsd = evals.eval(_cfg(NSD_ITEMS + ["neural_dataset=nsd", "log_expdata=true"]))
    syn = evals.eval(_cfg(NSD_ITEMS + ["neural_dataset=nsd_synthetic", "log_expdata=true"]))
    assert len(nsd) == len(syn) == 4
    assert list(syn["layer"]) == list(nsd["layer"])  # region-major, subject-minor in both
    assert all(s == [] for s in syn["layer_selection_scores"])

    cfg = _cfg(NSD_ITEMS + ["neural_dataset=nsd_synthetic"])
    model = _model(cfg, dev)
    data = load_nsd_synthetic_test_data(cfg, [0, 1], ["V1", "hV4"])
    k = 0
    for region in ["V1", "hV4"]:
        for subj in [0, 1]:
            row = syn.iloc[k]
            k += 1
            acts, got = _exact(model, data["stimuli"], dev, row["layer"], data["test_ids"])
            assert got == data["test_ids"]
            resp = np.stack([data["neural"][region][subj][s] for s in data["test_ids"]])
            rdm = _gpu_rdm(dev)
            point, scores, _, _ = O.bootstrap_rsa(rdm(acts), rdm(resp), 12, 42)
            assert abs(row["score"] - point) <= 1e-12
            assert np.max(np.abs(np.asarray(row["bootstrap_scores"]) - scores)) <= 1e-12


# --------------------------------------------------------------------------- PCA reconstruction
def test_rsa_phase2_reconstruct_from_pcs_matches_oracle(dev):
    from visreps_amd import evals
    from visreps_amd.dataloaders.neural import load_synthetic_data

    items = ["synthetic.n_test=90", "synthetic.n_train=120", "n_select=60", "n_bootstrap=10",
             "region=[V1]", "subject_idx=[0]", "batchsize=64", "reconstruct_from_pcs=true", "pca_k=3"]
    df = evals.eval(_cfg(items))
    plain = evals.eval(_cfg(items[:-2]))
    assert df.iloc[0]["layer"] == plain.iloc[0]["layer"]  # phase 1 is unchanged
    assert df.iloc[0]["score"] != plain.iloc[0]["score"]

    cfg = _cfg(items)
    model = _model(cfg, dev)
    data = load_synthetic_data(cfg, [0], ["V1"])
    test = data["stimuli"].subset(data["shared_test_ids"])
    acts, _ = _exact(model, test, dev, df.iloc[0]["layer"], data["shared_test_ids"])
    rec = P.reconstruct_from_pcs(acts, 3).astype(np.float32)
    resp = np.stack([data["neural"]["V1"][0]["test"][s] for s in data["shared_test_ids"]])
    point, scores, _, _ = O.bootstrap_rsa(O.compute_rdm(rec), O.compute_rdm(resp), 10, 42)
    # the reconstruction is fp64 on both sides; the RDMs are float32 numpy vs MFMA
    dp = abs(df.iloc[0]["score"] - point)
    db = float(np.max(np.abs(np.asarray(df.iloc[0]["bootstrap_scores"]) - scores)))
    record_margin("reconstruct_from_pcs_vs_oracle", n=len(resp), dspearman_point=dp, dspearman_boot=db)
    assert dp < TOL_SMALL_N and db < TOL_SMALL_N
