"""argparse.ArgumentParser with a "--config <yaml>" option whose keys become defaults —
espnet2/utils/config_argparse.py:7-47.  As in the reference: one config file, an unknown
key is an error, values are not type-checked, command-line options override the file."""
from __future__ import annotations

import argparse
from pathlib import Path

import yaml


class ArgumentParser(argparse.ArgumentParser):
    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.add_argument("--config", help="Give config file in yaml format")

    def parse_known_args(self, args=None, namespace=None):
        first, _ = super().parse_known_args(args, namespace)
        if first.config is not None:
            path = Path(first.config)
            if not path.exists():
                self.error(f"No such file: {first.config}")
            with path.open("r", encoding="utf-8") as f:
                conf = yaml.safe_load(f)
            if not isinstance(conf, dict):
                self.error(f"Config file has non dict value: {first.config}")
            known = {a.dest for a in self._actions}
            for key in conf:
                if key not in known:
                    self.error(f"unrecognized arguments: {key} (from {first.config})")
            self.set_defaults(**conf)
        return super().parse_known_args(args, namespace)
