"""Import-only stand-in for `typeguard` (absent from this image).

Only used by oracle/make_goldens.py when importing the reference to capture
golden vectors; the reference calls `assert check_argument_types()`.
"""


def check_argument_types(*a, **k):
    return True


def check_return_type(*a, **k):
    return True


def check_type(*a, **k):
    return None


def typechecked(fn=None, **k):
    return fn if fn is not None else (lambda f: f)
