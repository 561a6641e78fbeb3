"""CLI entry point: python -m visreps_amd.run --mode eval [--config F] [--override k=v ...]

Mirrors visreps/run.py: the base config is configs/<mode>/base.json, dotlist overrides
are applied by utils.load_config, validated by utils.validate_config, then dispatched.
Training (--mode train) is not part of this build (SURVEY.md §8 scope) and exits with an
error."""
from __future__ import annotations

import argparse
import sys

from . import utils


def main(argv=None) -> int:
    parser = argparse.ArgumentParser(description="visreps_amd evaluation (MI355X RSA path)")
    parser.add_argument("--mode", choices=["train", "eval"], default="eval")
    parser.add_argument("--config", default=None)
    parser.add_argument("--override", nargs="*", default=[])
    parser.add_argument("--verbose", "-v", action="store_true")
    args = parser.parse_args(argv)
    if args.mode == "train":
        print("visreps_amd: training is out of scope for this build; use --mode eval",
              file=sys.stderr)
        return 2
    overrides = list(args.override)
    if args.verbose:
        overrides.append("verbose=true")
    overrides.append(f"mode={args.mode}")
    cfg = utils.load_config(args.config or f"configs/{args.mode}/base.json", overrides)
    cfg = utils.validate_config(cfg)
    from . import evals  # imports torch + the HIP library only when evaluating

    evals.eval(cfg)
    return 0


if __name__ == "__main__":
    sys.exit(main())
