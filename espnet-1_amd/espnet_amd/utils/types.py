"""Argument value parsers of the reference's command line (espnet2/utils/types.py)."""
from __future__ import annotations

import re
from typing import Optional, Tuple, Union


def str2bool(value: str) -> bool:
    """"true"/"false" (any case) -> bool (types.py:7-9: strtobool semantics)."""
    v = str(value).strip().lower()
    if v in ("y", "yes", "t", "true", "on", "1"):
        return True
    if v in ("n", "no", "f", "false", "off", "0"):
        return False
    raise ValueError(f"invalid truth value {value!r}")


def _is_none(value: str) -> bool:
    return str(value).strip().lower() in ("none", "null", "nil")


def int_or_none(value: str) -> Optional[int]:
    return None if _is_none(value) else int(value)


def float_or_none(value: str) -> Optional[float]:
    return None if _is_none(value) else float(value)


def str_or_none(value: str) -> Optional[str]:
    return None if _is_none(value) else value


def str_or_int(value: str) -> Union[str, int]:
    try:
        return int(value)
    except ValueError:
        return value


def _strip(value: str) -> str:
    value = value.strip()
    if len(value) >= 2 and value[0] == value[-1] and value[0] in "'\"":
        value = value[1:-1]
    return value


def _split_tuple(value: str, n: int):
    v = value.strip()
    if v.startswith("(") and v.endswith(")"):
        v = v[1:-1]
    parts = [_strip(p) for p in v.split(",")]
    if len(parts) != n:
        raise TypeError(f"expected {n} comma-separated fields: {value}")
    return tuple(parts)


def str2pair_str(value: str) -> Tuple[str, str]:
    """"a,b" -> ("a", "b") (types.py:108-129)."""
    return _split_tuple(value, 2)


def str2triple_str(value: str) -> Tuple[str, str, str]:
    """"path,name,type" -> (path, name, type) (types.py:132-160)."""
    return _split_tuple(value, 3)


_SIZE = re.compile(r"^\s*([0-9.]+)\s*([kmgtpe]?)(i?)b?\s*$", re.I)


def parse_size(value) -> float:
    """humanfriendly.parse_size: "10MB" -> 1e7, "1GiB" -> 2**30, plain numbers as bytes."""
    if isinstance(value, (int, float)):
        return float(value)
    m = _SIZE.match(str(value))
    if not m:
        raise ValueError(f"invalid size: {value}")
    num, unit, binary = float(m.group(1)), m.group(2).lower(), m.group(3)
    exp = " kmgtpe".index(unit) if unit else 0
    return num * ((1024 if binary else 1000) ** exp)


def humanfriendly_parse_size_or_none(value) -> Optional[float]:
    return None if _is_none(value) else parse_size(value)
