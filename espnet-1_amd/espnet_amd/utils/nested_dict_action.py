"""argparse action that builds a dict from repeated "--x_conf key=value" options —
espnet2/utils/nested_dict_action.py:7-104 (same accepted syntaxes: key=<yaml>,
key.sub=<yaml>, a python dict literal or a yaml mapping).  Values are parsed with
yaml.safe_load / ast.literal_eval (no code is executed from the command line)."""
from __future__ import annotations

import argparse
import ast
import copy

import yaml


class NestedDictAction(argparse.Action):
    _syntax = ("Syntax:\n  {op} <key>=<yaml-string>\n  {op} <key>.<key2>=<yaml-string>\n"
               "  {op} <python-dict>\n  {op} <yaml-string>\n")

    def __init__(self, option_strings, dest, nargs=None, default=None, choices=None, required=False, help=None,
                 metavar=None):
        super().__init__(option_strings=option_strings, dest=dest, nargs=nargs, default=copy.deepcopy(default),
                         type=None, choices=choices, required=required, help=help, metavar=metavar)

    def __call__(self, parser, namespace, values, option_strings=None):
        if "=" in values and not values.lstrip().startswith("{"):
            current = copy.deepcopy(getattr(namespace, self.dest, None))
            if not isinstance(current, dict):
                current = {}
            key, value = values.split("=", maxsplit=1)
            if value.strip() != "":
                value = yaml.safe_load(value)
            node = current
            keys = key.split(".")
            for k in keys[:-1]:
                if not isinstance(node.get(k), dict):
                    node[k] = {}
                node = node[k]
            node[keys[-1]] = value
            setattr(namespace, self.dest, current)
            return
        try:
            value = ast.literal_eval(values)
        except (ValueError, SyntaxError):
            value = yaml.safe_load(values)
        if not isinstance(value, dict):
            raise argparse.ArgumentError(self, f"must be interpreted as dict: but got {values}\n"
                                               + self._syntax.format(op=option_strings))
        current = getattr(namespace, self.dest, None)
        if isinstance(current, dict):
            current.update(value)
        else:
            setattr(namespace, self.dest, value)
