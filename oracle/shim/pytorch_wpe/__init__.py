"""Import-only stand-in for `pytorch_wpe` (golden capture only): espnet2/asr/frontend/default.py
imports the WPE frontend module, which the single-channel path never calls."""


def wpe_one_iteration(*args, **kwargs):
    raise ImportError("pytorch_wpe is not available in this image")


def get_power(*args, **kwargs):
    raise ImportError("pytorch_wpe is not available in this image")


def get_correlations(*args, **kwargs):
    raise ImportError("pytorch_wpe is not available in this image")


def get_filter_matrix_conj(*args, **kwargs):
    raise ImportError("pytorch_wpe is not available in this image")


def perform_filter_operation(*args, **kwargs):
    raise ImportError("pytorch_wpe is not available in this image")
