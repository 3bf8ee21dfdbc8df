"""Placeholder submodule (golden capture only; never called on the ASR path)."""
