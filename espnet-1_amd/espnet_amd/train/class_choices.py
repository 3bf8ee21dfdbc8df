"""ClassChoices — espnet2/train/class_choices.py:9-92: a registry mapping a lower-cased
name to a class, with the reference's --<name> / --<name>_conf command-line options and
its type_check (every registered class must subclass it, :46-49)."""
from __future__ import annotations

from typing import Mapping, Optional, Tuple

from ..utils.nested_dict_action import NestedDictAction
from ..utils.types import str_or_none


class ClassChoices:
    def __init__(self, name: str, classes: Mapping[str, type], type_check: type = None, default: str = None,
                 optional: bool = False):
        self.name = name
        self.base_type = type_check
        self.classes = {k.lower(): v for k, v in classes.items()}
        if any(k in self.classes for k in ("none", "nil", "null")):
            raise ValueError('"none", "nil", and "null" are reserved.')
        if type_check is not None:
            for v in self.classes.values():
                if not issubclass(v, type_check):
                    raise ValueError(f"must be {type_check.__name__}, but got {v}")
        self.default = default
        self.optional = optional or default is None

    def choices(self) -> Tuple[Optional[str], ...]:
        return tuple(self.classes) + ((None,) if self.optional else ())

    def get_class(self, name: Optional[str]) -> Optional[type]:
        if name is None or (self.optional and str(name).lower() in ("none", "null", "nil")):
            return None
        key = str(name).lower()
        if key not in self.classes:
            raise ValueError(f"--{self.name} must be one of {self.choices()}: --{self.name} {key}")
        return self.classes[key]

    def add_arguments(self, parser):
        parser.add_argument(f"--{self.name}", type=lambda x: str_or_none(x.lower()), default=self.default,
                            choices=self.choices(), help=f"The {self.name} type")
        parser.add_argument(f"--{self.name}_conf", action=NestedDictAction, default=dict(),
                            help=f"The keyword arguments for {self.name}")
