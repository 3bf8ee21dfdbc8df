"""Import-only stand-in for `librosa`: any attribute use raises (golden capture only)."""


def __getattr__(name):
    raise ImportError(f"librosa.{name} is not available in this image")
