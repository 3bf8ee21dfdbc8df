"""Language models for shallow fusion in decoding (espnet2/lm)."""
from .transformer_lm import TransformerLM  # noqa: F401
