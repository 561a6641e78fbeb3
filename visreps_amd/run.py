"""Command line: ``python -m visreps_amd.run --mode eval [--config F] [--override k=v ...]``.

Same contract as visreps/run.py: configs/<mode>/base.json (or --config) is loaded, the
dotlist overrides are applied (utils.load_config) and checked (utils.validate_config),
and the eval entry point runs. Only ``eval`` is on this build's path; the
``train`` mode is accepted by the parser and refused with exit status 2.
"""
from __future__ import annotations

import argparse
import sys
from typing import List, Optional

from . import utils

_MODES = ("train", "eval")


def _parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="visreps_amd.run",
                                 description="visreps_amd evaluation (MI355X RSA path)")
    ap.add_argument("--mode", choices=_MODES, default="eval")
    ap.add_argument("--config", default=None, help="JSON config (default configs/<mode>/base.json)")
    ap.add_argument("--override", nargs="*", default=[], metavar="KEY=VALUE")
    ap.add_argument("--verbose", "-v", action="store_true")
    return ap


def _config_for(mode: str, path: Optional[str], dotlist: List[str], verbose: bool):
    items = [*dotlist, *(["verbose=true"] if verbose else []), f"mode={mode}"]
    return utils.validate_config(utils.load_config(path or f"configs/{mode}/base.json", items))


def main(argv=None) -> int:
    ns = _parser().parse_args(argv)
    if ns.mode != "eval":
        sys.stderr.write("visreps_amd: training is out of scope for this build; use --mode eval\n")
        return 2
    cfg = _config_for(ns.mode, ns.config, list(ns.override), ns.verbose)
    from . import evals  # torch and the HIP library load only for an actual evaluation

    evals.eval(cfg)
    return 0


if __name__ == "__main__":
    sys.exit(main())
