"""`--mode eval` drop-in (evals.eval / run CLI) on the synthetic NSD-shaped source.

CPU: CLI argument handling, config validation, loader ordering (string order for phase
1, int order for shared test IDs, as neural.py:170/:474).
GPU: eval() end to end at small size; the phase-2 point estimate and bootstrap are then
re-derived with the CPU oracle from the same exact activations: to 1e-12 on the eval's own
RDMs, and to the north-star 1e-5 on the oracle's numpy RDMs at n = 256 (configs[0]'s N). At
n = 96 the two fp32 RDMs' last-bit differences move near-tied ranks by 1.2e-5 of rho
(measured, profiles/r3_parity_margins.jsonl): each flip among M' = 3,655 pairs moves rho by up
to 12 / M'^2 ~ 1e-6, and the effect shrinks as 1 / M' with n."""
import numpy as np
import pytest
import torch

from visreps_amd import utils
from visreps_amd.run import main
from conftest import record_margin

# |dSpearman| between the product and the all-oracle path at these small n (each side builds
# its own RDMs): the north-star bound, with the measured values logged by record_margin
TOL_SMALL_N = 1e-5


def _cfg(**over):
    items = ["synthetic.n_test=256", "synthetic.n_train=160", "n_select=80", "n_bootstrap=20",
             "region=[V1,hV4]", "subject_idx=[0]", "batchsize=64"]
    items += [f"{k}={v}" for k, v in over.items()]
    cfg = utils.load_config("configs/eval/base.json", items + ["mode=eval"])
    return utils.validate_config(cfg)


def test_cli_train_mode_refused(capsys):
    assert main(["--mode", "train"]) == 2
    assert "out of scope" in capsys.readouterr().err


def test_config_synthetic_defaults():
    cfg = _cfg()
    assert cfg.neural_dataset == "synthetic" and cfg.random_init is True
    assert cfg.region == ["V1", "hV4"] and cfg.subject_idx == [0]
    assert cfg.synthetic["n_test"] == 256


def test_config_rejects_bad_compare_method():
    with pytest.raises(AssertionError):
        _cfg(compare_method="cosine")


def test_loader_orders():
    from visreps_amd.dataloaders.neural import StimulusLoader, SyntheticStimuli

    st = SyntheticStimuli({str(i): i for i in range(12)}, 1, "cpu")
    ids = [k for _, ks in StimulusLoader(st, 5) for k in ks]
    assert ids == sorted(ids, key=str) and ids[:4] == ["0", "1", "10", "11"]
    imgs, _ = next(iter(StimulusLoader(st, 5)))
    assert imgs.shape == (5, 3, 224, 224)


def test_loader_images_match_generator():
    from visreps_amd.dataloaders import synthetic as syn
    from visreps_amd.dataloaders.neural import SyntheticStimuli

    st = SyntheticStimuli({str(i): i for i in range(130)}, 3, "cpu")
    got = st.images([129, 0, 64, 5])
    ref = syn.make_images(range(0, 192), seed=3, device="cpu")
    assert torch.equal(got, ref[[129, 0, 64, 5]])


@pytest.mark.gpu
def test_eval_end_to_end_matches_oracle(dev):
    from oracle import rsa_oracle as O
    from visreps_amd import evals
    from visreps_amd.dataloaders.neural import _make_loader, load_synthetic_data
    from visreps_amd.models import utils as mutils

    cfg = _cfg()
    df = evals.eval(cfg)
    assert len(df) == 2
    assert set(df.columns) >= {"layer", "compare_method", "score", "ci_low", "ci_high",
                               "analysis", "layer_selection_scores", "bootstrap_scores"}
    for _, row in df.iterrows():
        sel = row["layer_selection_scores"]
        assert len(sel) == 14
        best = max(range(len(sel)), key=lambda i: (sel[i]["score"], -i))
        assert sel[best]["layer"] == row["layer"]
        assert len(row["bootstrap_scores"]) == 20 and row["ci_low"] <= row["ci_high"]

    # oracle re-derivation of phase 2 from the same exact activations
    cfg2 = _cfg()
    cfg2 = evals._load_cfg(cfg2)
    model = mutils.configure_feature_extractor(cfg2, mutils.load_model(cfg2, dev))
    data = load_synthetic_data(cfg2, [0], ["V1", "hV4"])
    test = data["stimuli"].subset(data["shared_test_ids"])
    for i, region in enumerate(["V1", "hV4"]):
        layer = df.iloc[i]["layer"]
        acts, got_ids = mutils.extract_single_layer(model, _make_loader(test, None, 64, 0), dev, layer,
                                                    data["shared_test_ids"])
        assert got_ids == data["shared_test_ids"]
        resp = np.stack([data["neural"][region][0]["test"][s] for s in data["shared_test_ids"]])
        # (a) the eval's own RDMs (same kernel, same rows) through the oracle's scipy
        #     Spearman + RandomState bootstrap: the Spearman path is exact
        from visreps_amd.analysis import rsa as R
        g_m = R.compute_rdm(acts.to(dev)).cpu().numpy()
        g_n = R.compute_rdm(torch.from_numpy(resp.astype(np.float32)).to(dev)).cpu().numpy()
        point, scores, lo, hi = O.bootstrap_rsa(g_m, g_n, n_bootstrap=20, seed=42)
        assert abs(df.iloc[i]["score"] - point) <= 1e-12
        assert np.max(np.abs(np.asarray(df.iloc[i]["bootstrap_scores"]) - scores)) <= 1e-12
        # percentiles of score vectors equal to 1e-12 (the engine's exact-integer statistic vs
        # scipy's float ranks differ in the last bits)
        assert abs(df.iloc[i]["ci_low"] - lo) <= 1e-12 and abs(df.iloc[i]["ci_high"] - hi) <= 1e-12
        # (b) fully oracle RDMs: entries within 1e-5, rho within the north-star 1e-5 (the
        #     bound at the bench's own N = 10k: tests/test_benchsize.py, ~1e-7 measured)
        m_rdm = O.compute_rdm(acts.numpy())
        n_rdm = O.compute_rdm(resp.astype(np.float32))
        assert np.max(np.abs(m_rdm - g_m)) < 1e-5 and np.max(np.abs(n_rdm - g_n)) < 1e-5
        point, scores, lo, hi = O.bootstrap_rsa(m_rdm, n_rdm, n_bootstrap=20, seed=42)
        dp = abs(df.iloc[i]["score"] - point)
        db = float(np.max(np.abs(np.asarray(df.iloc[i]["bootstrap_scores"]) - scores)))
        record_margin("eval_rsa_vs_oracle_rdms", n=len(resp), dspearman_point=dp, dspearman_boot=db,
                      rdm_err_model=float(np.max(np.abs(m_rdm - g_m))), rdm_err_neural=float(np.max(np.abs(n_rdm - g_n))))
        assert dp < TOL_SMALL_N and db < TOL_SMALL_N


@pytest.mark.gpu
def test_eval_encoding_score_end_to_end(dev):
    # evals._eval_encoding (evals.py:551-591): per (region, subject) train/test alignment on
    # the SRP activations -> compute_encoding_score; record layout of the reference
    from visreps_amd import evals

    cfg = _cfg(analysis="encoding_score", bootstrap="true")
    df = evals.eval(cfg)
    assert len(df) == 2
    for _, row in df.iterrows():
        assert row["analysis"] == "encoding_score" and row["compare_method"] == "pearson"
        sel = row["layer_selection_scores"]
        assert len(sel) == 14 and row["layer"] in [s["layer"] for s in sel]
        assert len(row["bootstrap_scores"]) == 20
        assert row["ci_low"] <= row["ci_high"] and np.isfinite(row["score"])
