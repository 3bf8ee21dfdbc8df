"""Import-only stand-in for `humanfriendly` (golden capture only)."""


def format_timespan(x, *a, **k):
    return f"{x}s"


def format_size(x, *a, **k):
    return f"{x}B"


def parse_size(x, *a, **k):
    return int(float(str(x).rstrip("BbKkMmGg") or 0))
