"""CPU-side checks of the native library and host logic (no GPU compute calls).

* every symbol declared in include/visreps_hip.h is exported by libvisreps_hip.so
* the native legacy-MT19937 stream is bit-exact against numpy.random.RandomState
* the native percentile equals numpy.percentile
* config / results-DB mirrors behave like the reference (utils.py)
"""
import json
import os
import re
import sqlite3

import numpy as np
import pandas as pd
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_header_symbols_exported():
    from visreps_amd import _lib

    header = open(os.path.join(ROOT, "include", "visreps_hip.h")).read()
    declared = set(re.findall(r"^\s*(?:[\w\s\*]+?)\b(vr_\w+)\s*\(", header, flags=re.M))
    assert declared, "no declarations parsed"
    lib = _lib.lib()
    for name in sorted(declared):
        assert hasattr(lib, name), f"{name} not exported"
    assert declared == set(_lib.EXPORTED_SYMBOLS)
    assert lib.vr_version() >= 100


@pytest.mark.parametrize("seed", [0, 1, 42, 99, 2**32 - 1])
def test_legacy_choice_bit_exact(seed):
    from visreps_amd.analysis._random import LegacyRandomState

    mine, ref = LegacyRandomState(seed), np.random.RandomState(seed)
    for n, k in [(10, 9), (50, 45), (256, 230), (1000, 900), (10000, 9000), (7, 0), (1, 1)]:
        a = mine.choice(n, size=k, replace=False)
        b = ref.choice(n, size=k, replace=False)
        assert a.dtype == b.dtype and np.array_equal(a, b)
    assert np.array_equal(mine.permutation(1854), ref.permutation(1854))


def test_raw_mt_stream_matches_numpy():
    from visreps_amd.analysis._random import LegacyRandomState

    from numpy.random import MT19937

    mine = LegacyRandomState(5489).random_u32(2000)
    bg = MT19937()
    bg._legacy_seeding(5489)  # RandomState(seed)'s init_genrand seeding
    assert np.array_equal(mine, bg.random_raw(2000).astype(np.uint32))


def test_bootstrap_indices_cache_and_stream():
    from visreps_amd.analysis._random import bootstrap_indices

    b = bootstrap_indices(42, 300, 270, 25)
    ref = np.random.RandomState(42)
    for i in range(25):
        assert np.array_equal(b[i], ref.choice(300, size=270, replace=False))
    assert bootstrap_indices(42, 300, 270, 25) is b
    assert not b.flags.writeable


@pytest.mark.parametrize("n,k,draws", [(1024, 921, 20), (3001, 2700, 37), (10000, 9000, 40), (1500, 1, 9)])
def test_draw_bootstrap_indices_threaded_path(n, k, draws):
    """vr_legacy_choice splits many draws over threads (sequential accept/reject replay,
    then permutations from the recorded generator states): bit-exact vs RandomState."""
    from visreps_amd.analysis._random import draw_bootstrap_indices
    rs = np.random.RandomState(42)
    ref = np.stack([rs.choice(n, k, replace=False) for _ in range(draws)]).astype(np.int32)
    np.testing.assert_array_equal(draw_bootstrap_indices(42, n, k, draws), ref)


def test_choice_errors():
    from visreps_amd.analysis._random import LegacyRandomState

    with pytest.raises(ValueError):
        LegacyRandomState(1).choice(5, size=6, replace=False)
    with pytest.raises(ValueError):
        LegacyRandomState(-1)


def test_percentile_matches_numpy():
    from visreps_amd.analysis.rsa import percentile

    rng = np.random.RandomState(0)
    for n in [1, 2, 3, 10, 999, 1000]:
        x = rng.randn(n)
        for q in [0, 2.5, 25, 50, 97.5, 100]:
            assert percentile(x, q) == np.percentile(x, q)
    x = rng.randn(10)
    x[3] = np.nan
    assert np.isnan(percentile(x, 50))


def test_config_two_pass_override(tmp_path):
    from visreps_amd.utils import load_config

    base = {
        "mode": "eval", "load_model_from": "checkpoint", "seed": 1, "cfg_id": 4,
        "checkpoint": {"checkpoint_dir": "/x", "checkpoint_model": "m.pth"},
        "torchvision": {"model_name": "AlexNet", "pretrained_dataset": "imagenet1k"},
        "region": ["V1"], "subject_idx": [0], "bootstrap": False,
    }
    p = tmp_path / "base.json"
    p.write_text(json.dumps(base))
    cfg = load_config(p, ["bootstrap=true", "checkpoint_dir=/y", "subject_idx=[0,1]", "mode=eval"])
    assert cfg.bootstrap is True and cfg.subject_idx == [0, 1]
    assert cfg.checkpoint_dir == "/y" and "checkpoint" not in cfg and "torchvision" not in cfg
    cfg2 = load_config(p, ["load_model_from=torchvision", "mode=eval"])
    assert cfg2.model_name == "AlexNet" and "cfg_id" not in cfg2


def test_config_verifier():
    from visreps_amd.utils import Config, validate_config

    good = Config({"mode": "eval", "seed": 1, "neural_dataset": "nsd", "subject_idx": 0,
                   "region": "V1", "compare_method": "spearman", "analysis": "rsa",
                   "return_nodes": ["conv1"], "load_model_from": "torchvision"})
    cfg = validate_config(good)
    assert cfg.subject_idx == [0] and cfg.region == ["V1"]
    for bad in [{"seed": 4}, {"region": "IT"}, {"compare_method": "pearson"}, {"subject_idx": 9}]:
        c = Config(dict(good))
        c.update(bad)
        with pytest.raises(AssertionError):
            validate_config(c)


def test_results_db_roundtrip(tmp_path, monkeypatch):
    import visreps_amd.utils as vu

    monkeypatch.setattr(vu, "_RESULTS_DB_PATH", tmp_path / "r.db")
    cfg = vu.Config({"seed": 1, "epoch": 20, "region": "V1", "subject_idx": 0,
                     "neural_dataset": "nsd", "cfg_id": 1000, "pca_labels": False,
                     "analysis": "rsa", "compare_method": "spearman", "model_name": "AlexNet"})
    df = pd.DataFrame([{"layer": "fc1_pre", "compare_method": "spearman", "score": 0.25,
                        "ci_low": 0.2, "ci_high": 0.3, "analysis": "rsa",
                        "layer_selection_scores": [{"layer": "conv1", "score": 0.1},
                                                   {"layer": "fc1_pre", "score": 0.25}],
                        "bootstrap_scores": [0.2, 0.25, 0.3]}])
    vu.save_results(df, cfg)
    df2 = df.copy()
    df2.loc[0, "score"] = 0.3
    vu.save_results(df2, cfg)
    conn = sqlite3.connect(str(tmp_path / "r.db"))
    rows = pd.read_sql("SELECT * FROM results", conn)
    assert len(rows) == 1 and rows.iloc[0]["score"] == pytest.approx(0.3)
    assert len(pd.read_sql("SELECT * FROM layer_selection_scores", conn)) == 2
    bs = pd.read_sql("SELECT * FROM bootstrap_distributions", conn)
    assert json.loads(bs.iloc[0]["scores"]) == [0.2, 0.25, 0.3]
    assert rows.iloc[0]["run_id"] == vu._compute_run_id(cfg)
    conn.close()
