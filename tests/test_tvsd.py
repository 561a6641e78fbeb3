"""`neural_dataset=tvsd` through the two-phase RSA path (reference evals.py:189-190 ->
_eval_rsa :222-400; data contract neural.py:393-460) on the TVSD-shaped synthetic source:
V1 / V4 / IT MUA of two monkeys, ~22k train stimuli per subject (phase 1 draws n_select =
1000 of them, evals.py:235-263) and 100 shared test stimuli sorted as strings.

CPU: config validation and the loader contract. GPU: eval() at the default TVSD sizes,
re-derived with the CPU oracle -- phase 1 from the product's own SRP activations
(RandomState(42).choice over the string-ordered train rows, numpy RDMs, scipy Spearman,
first strict maximum), phase 2 on the eval's own RDMs (exact: 1e-12)."""
import numpy as np
import pytest
import torch

from conftest import record_margin
from visreps_amd import utils

TOL = 1e-5  # north-star |dSpearman|; each side builds its own selection RDMs


def _cfg(items=()):
    base = ["neural_dataset=tvsd", "region=[V1,V4,IT]", "subject_idx=[0,1]", "n_bootstrap=20",
            "batchsize=128", "bootstrap=true"]
    return utils.validate_config(utils.load_config("configs/eval/base.json", base + list(items) + ["mode=eval"]))


def test_tvsd_config_validation():
    cfg = _cfg()
    assert cfg.region == ["V1", "V4", "IT"] and cfg.subject_idx == [0, 1]
    with pytest.raises(AssertionError, match="TVSD"):
        _cfg(["region=[V2]"])
    with pytest.raises(AssertionError, match="monkey"):
        _cfg(["subject_idx=[2]"])


def test_tvsd_loader_contract():
    from visreps_amd.dataloaders.neural import TVSD_VOXELS, load_tvsd_synthetic

    cfg = _cfg(["synthetic.tvsd_n_train=40", "synthetic.tvsd_n_test=12"])
    d = load_tvsd_synthetic(cfg, [0, 1], ["V1", "IT"])
    assert d["regions"] == ["V1", "IT"] and d["subjects"] == [0, 1]
    test_ids = d["shared_test_ids"]
    assert len(test_ids) == 12 and test_ids == sorted(test_ids)  # string order (neural.py:453)
    for r in ("V1", "IT"):
        for s in (0, 1):
            tr, te = d["neural"][r][s]["train"], d["neural"][r][s]["test"]
            assert len(tr) == 40 and set(te) == set(test_ids) and not set(tr) & set(te)
            assert next(iter(tr.values())).shape == (TVSD_VOXELS[r],)
    assert set(d["stimuli"]) == set(d["neural"]["V1"][0]["train"]) | set(test_ids)
    a, b = d["neural"]["V1"][0]["train"], d["neural"]["V1"][1]["train"]
    k = next(iter(a))
    assert not np.array_equal(a[k], b[k])  # per-subject responses


@pytest.mark.gpu
def test_tvsd_eval_matches_oracle(dev):
    from oracle import rsa_oracle as O
    from visreps_amd import evals
    from visreps_amd.analysis import rsa as R
    from visreps_amd.analysis.alignment import _align_stimulus_level
    from visreps_amd.dataloaders.neural import _make_loader, load_tvsd_synthetic
    from visreps_amd.models import utils as mutils

    cfg = _cfg()
    df = evals.eval(cfg)
    assert len(df) == 6  # region-major, subject-minor
    cfg2 = evals._load_cfg(_cfg())
    model = mutils.configure_feature_extractor(cfg2, mutils.load_model(cfg2, dev))
    data = load_tvsd_synthetic(cfg2, [0, 1], ["V1", "V4", "IT"])
    assert len(data["neural"]["V1"][0]["train"]) == 22248 and len(data["shared_test_ids"]) == 100
    acts, ids = mutils.get_activations(model, _make_loader(data["stimuli"], None, 128, 0), dev,
                                       keep_on_device=True, srp_seed=cfg2.get("srp_seed"),
                                       srp_cache_dir=cfg2.get("srp_cache_dir", "model_checkpoints/srp_cache"))
    test = data["stimuli"].subset(data["shared_test_ids"])
    k = 0
    for region in ["V1", "V4", "IT"]:
        for subj in [0, 1]:
            row = df.iloc[k]
            k += 1
            # phase 1 (evals.py:249-287) in the oracle
            tr_acts, tr_neural, _ = _align_stimulus_level(acts, data["neural"][region][subj]["train"], ids)
            assert tr_neural.size(0) == 22248
            sel = np.random.RandomState(42).choice(22248, 1000, replace=False)
            n_rdm = O.compute_rdm(tr_neural.cpu().numpy()[sel])
            scores = [O.compute_rdm_correlation(O.compute_rdm(a.cpu().numpy()[sel]), n_rdm, "Spearman")
                      for a in tr_acts.values()]
            got = row["layer_selection_scores"]
            assert [g["layer"] for g in got] == list(tr_acts)
            d = float(np.max(np.abs(np.array([g["score"] for g in got]) - np.array(scores))))
            record_margin("tvsd_phase1_vs_oracle", region=region, subject=subj, n_train=22248, dspearman=d)
            assert d < TOL
            best = int(np.argmax(scores))
            srt = np.sort(scores)
            if srt[-1] - srt[-2] > 2 * TOL:  # not a near-tie: the choice must agree
                assert row["layer"] == list(tr_acts)[best]
            # phase 2 + scoring on the eval's own RDMs (evals.py:333-373)
            ex, got_ids = mutils.extract_single_layer(model, _make_loader(test, None, 128, 0), dev,
                                                      row["layer"], data["shared_test_ids"], keep_on_device=True)
            assert got_ids == data["shared_test_ids"]
            resp = np.stack([data["neural"][region][subj]["test"][s] for s in data["shared_test_ids"]])
            g_m = R.compute_rdm(ex).cpu().numpy()
            g_n = R.compute_rdm(torch.from_numpy(resp).to(dev)).cpu().numpy()
            point, boots, lo, hi = O.bootstrap_rsa(g_m, g_n, n_bootstrap=20, seed=42)
            assert abs(row["score"] - point) <= 1e-12
            assert np.max(np.abs(np.asarray(row["bootstrap_scores"]) - boots)) <= 1e-12
            assert abs(row["ci_low"] - lo) <= 1e-12 and abs(row["ci_high"] - hi) <= 1e-12
