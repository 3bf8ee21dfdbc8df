"""Import-only stand-in for `librosa` (golden capture only; librosa is not in this image).

`librosa.filters.mel` is restated (oracle/shim/librosa/filters.py) so the reference's LogMel
(espnet2/layers/log_mel.py:51) can be constructed; every other attribute raises."""
from . import filters  # noqa: F401


def __getattr__(name):
    raise ImportError(f"librosa.{name} is not available in this image")
