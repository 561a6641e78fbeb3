"""Console, config and results-DB helpers of the eval path (reference: visreps/utils.py).

Only the parts `python -m visreps.run --mode eval` needs are mirrored:
  * rprint / console                          utils.py:57-73
  * Config: attribute-access dict with OmegaConf-style dotlist overrides (omegaconf is
    not installed here; values are parsed as YAML like OmegaConf.from_dotlist does)
  * load_config / merge_nested_config         utils.py:467-507 (two-pass override merge)
  * ConfigVerifier (eval part) / validate_config  utils.py:461-464, 582-755
  * results DB: _IDENTITY_FIELDS, _compute_run_id, _init_db, save_results  utils.py:300-458
"""
from __future__ import annotations

import copy
import hashlib
import json
import sqlite3
from pathlib import Path
from typing import Any, Iterable

import yaml

try:  # rich is optional; plain print keeps the same text
    from rich.console import Console
    from rich.theme import Theme

    console = Console(
        theme=Theme(
            {
                "info": "bold white",
                "success": "green",
                "warning": "bold yellow",
                "error": "bold red",
                "highlight": "bold magenta",
                "setup": "cyan",
            }
        )
    )
    rprint = console.print
except Exception:  # pragma: no cover
    console = None

    def rprint(*args, style=None, **kwargs):  # noqa: ARG001
        print(*args)


# -----------------------------------------------------------------------------
# Config
# -----------------------------------------------------------------------------
class Config(dict):
    """dict with attribute access; nested dicts become Config (DictConfig stand-in)."""

    def __init__(self, *args, **kwargs):
        super().__init__()
        for k, v in dict(*args, **kwargs).items():
            self[k] = v

    @staticmethod
    def _wrap(v):
        if isinstance(v, Config):
            return v
        if isinstance(v, dict):
            return Config(v)
        if isinstance(v, (list, tuple)):
            return [Config._wrap(x) for x in v]
        return v

    def __setitem__(self, k, v):
        super().__setitem__(k, Config._wrap(v))

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError:
            raise AttributeError(k) from None

    def __setattr__(self, k, v):
        self[k] = v

    def __delattr__(self, k):
        try:
            del self[k]
        except KeyError:
            raise AttributeError(k) from None

    def __deepcopy__(self, memo):
        return Config(copy.deepcopy(dict(self), memo))

    def to_container(self) -> dict:
        def plain(v):
            if isinstance(v, dict):
                return {k: plain(x) for k, x in v.items()}
            if isinstance(v, list):
                return [plain(x) for x in v]
            return v

        return plain(self)

    def merge(self, other: dict) -> "Config":
        """OmegaConf.merge semantics for plain data: nested dicts merge, others replace."""
        out = copy.deepcopy(self)
        for k, v in other.items():
            if isinstance(v, dict) and isinstance(out.get(k), dict):
                out[k] = Config(out[k]).merge(v)
            else:
                out[k] = copy.deepcopy(v)
        return out


def _parse_value(text: str) -> Any:
    if text == "":
        return ""
    try:
        return yaml.safe_load(text)
    except yaml.YAMLError:
        return text


def from_dotlist(items: Iterable[str]) -> Config:
    """OmegaConf.from_dotlist: 'a.b=1' -> {'a': {'b': 1}}, values parsed as YAML."""
    out = Config()
    for item in items:
        if "=" not in item:
            raise ValueError(f"override '{item}' is not key=value")
        key, val = item.split("=", 1)
        node = out
        parts = key.strip().split(".")
        for p in parts[:-1]:
            if not isinstance(node.get(p), dict):
                node[p] = Config()
            node = node[p]
        node[parts[-1]] = _parse_value(val.strip())
    return out


def merge_nested_config(cfg: Config, source_key: str) -> None:
    """Lift cfg[source_key]'s entries to the root and drop the section (utils.py:467-474)."""
    if source_key not in cfg:
        return
    source = Config(cfg[source_key]).to_container()
    cfg.update(Config(source))
    del cfg[source_key]


def load_config(config_path, overrides=None) -> Config:
    """Base JSON + dotlist overrides applied twice around the nested-section flattening
    (utils.py:477-507)."""
    path = Path(config_path)
    if not path.exists():
        raise FileNotFoundError(f"Config file not found: {config_path}")
    cfg = Config(json.loads(path.read_text()))
    ov = from_dotlist(overrides) if overrides else None
    if ov:
        cfg = cfg.merge(ov)
    mode = cfg.get("mode")
    source_key = cfg.get("load_model_from") if mode == "eval" else cfg.get("model_class")
    if source_key:
        other = {
            "eval": {"torchvision": "checkpoint", "checkpoint": "torchvision"},
            "train": {"custom_model": "standard_model", "standard_model": "custom_model"},
        }[mode].get(source_key)
        if other and other in cfg:
            del cfg[other]
        merge_nested_config(cfg, source_key)
    if ov:
        cfg = cfg.merge(ov)
    if cfg.get("mode") == "eval" and cfg.get("load_model_from") == "torchvision":
        cfg.pop("cfg_id", None)
    if cfg.get("verbose", False):
        rprint(f"Final Configuration:\n{yaml.safe_dump(cfg.to_container())}\n")
    return cfg


def get_seed_letter(seed) -> str:
    """Seed 1-9 -> 'a'-'i' (utils.py:895-899)."""
    if not isinstance(seed, int) or seed < 1 or seed > 9:
        raise ValueError(f"Seed must be an integer between 1-9, got {seed}")
    return chr(ord("a") + seed - 1)


class ConfigVerifier:
    """Eval-mode validation (utils.py:510-755). Training validation is out of scope."""

    VALID_MODES = {"train", "eval"}
    VALID_MODEL_SOURCES = {"checkpoint", "torchvision"}
    VALID_ANALYSES = {"rsa", "encoding_score"}
    VALID_COMPARE_METHODS = {"spearman", "kendall"}
    VALID_NEURAL_DATASETS = {"nsd", "things-behavior", "tvsd", "nsd_synthetic", "synthetic"}
    NSD_REGIONS = {
        "early visual stream", "ventral visual stream", "V1", "V2", "V3", "hV4", "FFA", "PPA",
    }
    TVSD_REGIONS = {"V1", "V4", "IT"}

    def __init__(self, cfg: Config):
        self.cfg = cfg

    def verify(self) -> Config:
        if self.cfg.get("mode") not in self.VALID_MODES:
            raise AssertionError(f"Invalid mode: {self.cfg.get('mode')}")
        if self.cfg.mode == "train":
            raise AssertionError("training is not part of the MI355X RSA eval build")
        return self._verify_eval()

    @staticmethod
    def _as_list(v):
        return list(v) if isinstance(v, (list, tuple)) else [v]

    def _verify_eval(self) -> Config:
        cfg = self.cfg
        if cfg.get("seed") not in (1, 2, 3):
            raise AssertionError(f"Invalid seed: {cfg.get('seed')}")
        ds = str(cfg.neural_dataset).lower()
        if ds == "things-behavior":
            region, subj = cfg.get("region"), cfg.get("subject_idx")
            if region is not None and not (isinstance(region, str) and region.upper() == "N/A"):
                rprint(f"Region '{region}' provided for 'things-behavior' dataset. Setting to 'N/A'.",
                       style="warning")
                cfg.region = "N/A"
            if subj is not None and not (isinstance(subj, str) and subj.upper() == "N/A"):
                rprint(f"Subject index '{subj}' provided for 'things-behavior' dataset. Setting to 'N/A'.",
                       style="warning")
                cfg.subject_idx = "N/A"
        if ds in ("nsd", "nsd_synthetic"):
            cfg.subject_idx = self._as_list(cfg.subject_idx)
            for s in cfg.subject_idx:
                if not isinstance(s, int) or not 0 <= s < 8:
                    raise AssertionError(
                        f"Invalid subject index for NSD: {s}. Must be an integer in range [0, 7]")
            cfg.region = self._as_list(cfg.region)
            for r in cfg.region:
                if r not in self.NSD_REGIONS:
                    raise AssertionError(f"Invalid region for NSD: {r}. Must be one of {self.NSD_REGIONS}")
        if ds == "tvsd":
            cfg.subject_idx = self._as_list(cfg.subject_idx)
            for s in cfg.subject_idx:
                if not isinstance(s, int) or s not in (0, 1):
                    raise AssertionError(
                        f"Invalid subject_idx for TVSD: {s}. Must be 0 (monkey F) or 1 (monkey N)")
            cfg.region = self._as_list(cfg.region)
            for r in cfg.region:
                if r not in self.TVSD_REGIONS:
                    raise AssertionError(f"Invalid region for TVSD: {r}. Must be one of {self.TVSD_REGIONS}")
        if ds == "synthetic":
            cfg.subject_idx = self._as_list(cfg.get("subject_idx", 0))
            cfg.region = self._as_list(cfg.get("region", "V1"))
        compare_method = str(cfg.get("compare_method", "spearman")).lower()
        if compare_method not in self.VALID_COMPARE_METHODS:
            raise AssertionError(f"Invalid compare_method: {compare_method}")
        if str(cfg.analysis).lower() not in self.VALID_ANALYSES:
            raise AssertionError(f"Invalid analysis: {cfg.analysis}")
        if str(cfg.analysis).lower() == "encoding_score":
            if ds == "things-behavior":
                raise AssertionError(
                    "analysis=encoding_score is not supported for things-behavior "
                    "(behavioral embeddings have no voxels to predict). Use analysis=rsa instead.")
            if ds == "nsd_synthetic":
                raise AssertionError(
                    "analysis=encoding_score is not supported for nsd_synthetic. Use analysis=rsa instead.")
            cfg.compare_method = "pearson"
        rn = cfg.get("return_nodes")
        if rn is None or isinstance(rn, (str, int)) or not hasattr(rn, "__iter__"):
            raise AssertionError("return_nodes must be a list-like object")
        if not rn:
            raise AssertionError("return_nodes list cannot be empty")
        if cfg.get("load_model_from") not in self.VALID_MODEL_SOURCES:
            raise AssertionError(f"load_model_from must be in {self.VALID_MODEL_SOURCES}")
        if cfg.load_model_from == "checkpoint":
            if "torchvision" in cfg:
                raise AssertionError("torchvision key not allowed in checkpoint mode")
            if not cfg.get("random_init", False):
                ckpt = Path(f"{cfg.checkpoint_dir}/cfg{cfg.cfg_id}{get_seed_letter(cfg.seed)}/"
                            f"{cfg.checkpoint_model}")
                if not ckpt.exists():
                    raise AssertionError(f"Checkpoint not found: {ckpt}")
        return cfg


def validate_config(cfg: Config) -> Config:
    return ConfigVerifier(cfg).verify()


# -----------------------------------------------------------------------------
# Results DB (same schema and run_id as the reference so plotters read it unchanged)
# -----------------------------------------------------------------------------
_RESULTS_DB_PATH = Path("results.db")

_IDENTITY_FIELDS = (
    "seed", "epoch", "region", "subject_idx", "neural_dataset", "cfg_id",
    "pca_labels", "pca_n_classes", "pca_labels_folder", "checkpoint_dir",
    "analysis", "compare_method", "reconstruct_from_pcs", "pca_k", "model_name",
)


def _compute_run_id(cfg) -> str:
    """sha256[:12] of the identity fields (utils.py:307-312)."""
    identity = {f: cfg.get(f) for f in _IDENTITY_FIELDS}
    identity["subject_idx"] = str(identity.get("subject_idx"))
    raw = json.dumps(identity, sort_keys=True)
    return hashlib.sha256(raw.encode()).hexdigest()[:12]


def _init_db(db_path) -> sqlite3.Connection:
    db_path = Path(db_path)
    db_path.parent.mkdir(parents=True, exist_ok=True)
    conn = sqlite3.connect(str(db_path), timeout=10)
    conn.execute("PRAGMA journal_mode=WAL")
    conn.execute("PRAGMA busy_timeout=10000")
    conn.execute(
        """CREATE TABLE IF NOT EXISTS results (
            run_id TEXT NOT NULL, compare_method TEXT NOT NULL, layer TEXT NOT NULL,
            score REAL, ci_low REAL, ci_high REAL, analysis TEXT NOT NULL,
            seed INTEGER NOT NULL, epoch INTEGER NOT NULL, region TEXT, subject_idx TEXT,
            neural_dataset TEXT NOT NULL, cfg_id INTEGER, pca_labels BOOLEAN NOT NULL,
            pca_n_classes INTEGER, pca_labels_folder TEXT, model_name TEXT NOT NULL,
            checkpoint_dir TEXT, reconstruct_from_pcs BOOLEAN DEFAULT 0, pca_k INTEGER DEFAULT 1,
            UNIQUE(run_id, compare_method, layer))"""
    )
    conn.execute(
        """CREATE TABLE IF NOT EXISTS run_configs (
            run_id TEXT PRIMARY KEY, config_json TEXT NOT NULL,
            created_at TEXT DEFAULT (datetime('now')))"""
    )
    conn.execute(
        """CREATE TABLE IF NOT EXISTS layer_selection_scores (
            run_id TEXT NOT NULL, compare_method TEXT NOT NULL, layer TEXT NOT NULL,
            score REAL, UNIQUE(run_id, compare_method, layer))"""
    )
    conn.execute(
        """CREATE TABLE IF NOT EXISTS bootstrap_distributions (
            run_id TEXT NOT NULL, compare_method TEXT NOT NULL, scores TEXT,
            UNIQUE(run_id, compare_method))"""
    )
    conn.commit()
    return conn


def _get_float(row, col):
    import pandas as pd

    if col in row.index and pd.notna(row.get(col)):
        return float(row[col])
    return None


def save_results(df, cfg, timeout=60):  # noqa: ARG001
    """Persist one result table in the reference's long format (utils.py:381-458)."""
    run_id = _compute_run_id(cfg)
    conn = _init_db(_RESULTS_DB_PATH)
    container = cfg.to_container() if isinstance(cfg, Config) else dict(cfg)
    conn.execute("INSERT OR REPLACE INTO run_configs (run_id, config_json) VALUES (?, ?)",
                 (run_id, json.dumps(container)))
    for _, row in df.iterrows():
        method = row.get("compare_method", cfg.get("compare_method", "spearman"))
        score = _get_float(row, "score")
        if score is None:
            continue
        conn.execute(
            """INSERT OR REPLACE INTO results
               (run_id, compare_method, layer, score, ci_low, ci_high, analysis, seed, epoch,
                region, subject_idx, neural_dataset, cfg_id, pca_labels, pca_n_classes,
                pca_labels_folder, model_name, checkpoint_dir, reconstruct_from_pcs, pca_k)
               VALUES (?, ?, ?, ?, ?, ?, ?, ?, ?, ?, ?, ?, ?, ?, ?, ?, ?, ?, ?, ?)""",
            (
                run_id, method, row.get("layer"), score, _get_float(row, "ci_low"),
                _get_float(row, "ci_high"), row.get("analysis", cfg.get("analysis")),
                int(cfg.get("seed")), int(cfg.get("epoch", 0)), cfg.get("region"),
                str(cfg.get("subject_idx")), cfg.get("neural_dataset"), cfg.get("cfg_id"),
                bool(cfg.get("pca_labels")), cfg.get("pca_n_classes"),
                cfg.get("pca_labels_folder"), cfg.get("model_name"), cfg.get("checkpoint_dir"),
                bool(cfg.get("reconstruct_from_pcs", False)), cfg.get("pca_k", 1),
            ),
        )
    for _, row in df.iterrows():
        method = row.get("compare_method", cfg.get("compare_method", "spearman"))
        entries = row.get("layer_selection_scores")
        if isinstance(entries, list):
            for entry in entries:
                conn.execute(
                    """INSERT OR REPLACE INTO layer_selection_scores
                       (run_id, compare_method, layer, score) VALUES (?, ?, ?, ?)""",
                    (run_id, method, entry["layer"], float(entry["score"])),
                )
    for _, row in df.iterrows():
        method = row.get("compare_method", cfg.get("compare_method", "spearman"))
        bs = row.get("bootstrap_scores") if "bootstrap_scores" in row.index else None
        if isinstance(bs, list):
            conn.execute(
                """INSERT OR REPLACE INTO bootstrap_distributions
                   (run_id, compare_method, scores) VALUES (?, ?, ?)""",
                (run_id, method, json.dumps(bs)),
            )
    conn.commit()
    conn.close()
    rprint(f"Saved {len(df)} results to {_RESULTS_DB_PATH} (run_id={run_id})", style="success")
    return str(_RESULTS_DB_PATH)
