"""TransformerEncoder — drop-in for espnet2/asr/encoder/transformer_encoder.py:37-232
(BASELINE.json configs[0]: the Transformer-tiny of egs2/mini_an4).

Same constructor signature and state_dict layout (embed.conv.{0,2}, embed.out.0,
encoders.{i}.{self_attn,feed_forward,norm1,norm2}, after_norm); forward runs the HIP
path: Conv2dSubsampling with the absolute PositionalEncoding (subsampling.py:57-69 with
PositionalEncoding(odim, dropout_rate) — the reference passes the encoder's dropout_rate,
not positional_dropout_rate, to it) -> N x TransformerBlockFn -> after_norm.  Options the
ASR recipes do not use (other input layers, conv1d feed-forward, concat_after,
normalize_before=False, interCTC) raise NotImplementedError.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
from torch import nn

from ... import hip_ops as ops
from ..._lib import lib
from ...layers.common import LayerNormFn, multisequential_draw
from ...layers.conformer import MultiHeadedAttention, PositionwiseFeedForward
from ...layers.decoder import PositionalEncoding
from ...layers.subsampling import Conv2dSubsampling
from ...layers.transformer import TransformerEncoderLayer
from .conformer_encoder import AbsEncoder, TooShortUttError, _AfterNorm


class TransformerEncoder(AbsEncoder):
    def __init__(
        self,
        input_size: int,
        output_size: int = 256,
        attention_heads: int = 4,
        linear_units: int = 2048,
        num_blocks: int = 6,
        dropout_rate: float = 0.1,
        positional_dropout_rate: float = 0.1,
        attention_dropout_rate: float = 0.0,
        input_layer: Optional[str] = "conv2d",
        pos_enc_class=None,
        normalize_before: bool = True,
        concat_after: bool = False,
        positionwise_layer_type: str = "linear",
        positionwise_conv_kernel_size: int = 1,
        padding_idx: int = -1,
        interctc_layer_idx: List[int] = [],
        interctc_use_conditioning: bool = False,
    ):
        super().__init__()
        self._output_size = output_size
        if input_layer not in ("linear", "conv2d", "conv2d1", "conv2d2", "conv2d6", "conv2d8", "embed", None):
            raise ValueError("unknown input_layer: " + str(input_layer))
        if positionwise_layer_type not in ("linear", "conv1d", "conv1d-linear"):
            raise NotImplementedError("Support only linear or conv1d.")
        unsupported = []
        if input_layer != "conv2d":
            unsupported.append(f"input_layer={input_layer}")
        if positionwise_layer_type != "linear":
            unsupported.append(f"positionwise_layer_type={positionwise_layer_type}")
        if pos_enc_class is not None and pos_enc_class is not PositionalEncoding:
            unsupported.append("pos_enc_class")
        if not normalize_before or concat_after:
            unsupported.append("normalize_before=False/concat_after")
        if interctc_layer_idx:
            unsupported.append("interctc")
        if unsupported:
            raise NotImplementedError("espnet_amd TransformerEncoder implements the ASR recipes' "
                                      "configuration only; unsupported: " + ", ".join(unsupported))
        if output_size % 8:
            raise ValueError("output_size must be a multiple of 8 (16-B aligned MFMA operands)")
        self.embed = Conv2dSubsampling(input_size, output_size, dropout_rate,
                                       PositionalEncoding(output_size, dropout_rate))
        self.normalize_before = normalize_before
        layers = []
        for lnum in range(num_blocks):
            layers.append(TransformerEncoderLayer(
                output_size, MultiHeadedAttention(attention_heads, output_size, attention_dropout_rate),
                PositionwiseFeedForward(output_size, linear_units, dropout_rate, activation="relu"),
                dropout_rate, normalize_before, concat_after))
            layers[-1].layer_idx = lnum + 1
        self.encoders = nn.Sequential(*layers)
        self.after_norm = _AfterNorm(output_size, eps=1e-12)
        self.interctc_layer_idx = interctc_layer_idx
        self.interctc_use_conditioning = interctc_use_conditioning
        self.conditioning_layer = None

    def output_size(self) -> int:
        return self._output_size

    def arena_groups(self, prefix=""):
        g = []
        for i in range(len(self.encoders)):
            g += TransformerEncoderLayer.arena_groups(f"{prefix}encoders.{i}.")
        return g

    def bind(self, arena, prefix, cd, anchor):
        self.embed.bind(arena, prefix + "embed.", cd)
        self.embed._anchor = anchor
        for i, layer in enumerate(self.encoders):
            layer.bind(arena, f"{prefix}encoders.{i}.", cd)
        self.after_norm.bind(arena, prefix + "after_norm.", cd)
        self._cd = cd

    def forward(self, xs_pad: torch.Tensor, ilens: torch.Tensor, prev_states=None, ctc=None,
                seed: int = 0) -> Tuple[torch.Tensor, torch.Tensor, Optional[torch.Tensor]]:
        """transformer_encoder.py:184-232.  xs_pad (B,T,F) f32 on the GPU, ilens (B,) int64."""
        B, T, _ = xs_pad.shape
        if T < 7:  # check_short_utt, subsampling.py:31-43
            raise TooShortUttError(f"has {T} frames and is too short for subsampling "
                                   f"(it needs more than 7 frames), return empty results", T, 7)
        xs_pad = xs_pad.contiguous()
        olens = torch.empty(B, dtype=torch.long, device=xs_pad.device)
        lib.ea_subsample_lens(B, T, ilens.data_ptr(), olens.data_ptr(), ops.stream())
        x = self.embed(xs_pad, seed)
        multisequential_draw(len(self.encoders))
        for layer in self.encoders:
            x = layer(x, olens, seed)
        x = LayerNormFn.apply(x, self.after_norm)
        return x, olens, None
