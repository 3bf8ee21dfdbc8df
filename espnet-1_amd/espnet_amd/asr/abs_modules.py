"""Abstract module types the ASR registries check against (ClassChoices type_check,
espnet2/tasks/asr.py:88-188): espnet2/asr/frontend/abs_frontend.py, specaug/abs_specaug.py,
layers/abs_normalize.py."""
from __future__ import annotations

from torch import nn


class AbsFrontend(nn.Module):
    def output_size(self) -> int:
        raise NotImplementedError


class AbsSpecAug(nn.Module):
    pass


class AbsNormalize(nn.Module):
    pass
