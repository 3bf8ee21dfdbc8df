"""ConformerEncoder — drop-in for espnet2/asr/encoder/conformer_encoder.py:49-377.

Same constructor signature, option validation and state_dict layout; forward runs the
HIP path: Conv2dSubsampling (SubsampleFn) -> N x ConformerBlockFn -> after_norm.
Only the configuration the reference's ASR recipes train (input_layer conv2d,
rel_pos_type latest, rel_pos / rel_selfattn, macaron, conv module, normalize_before) is
implemented; other choices raise NotImplementedError instead of silently diverging.
"""
from __future__ import annotations

from typing import List, Optional, Tuple, Union

import torch
from torch import nn

from ...layers.common import LayerNormFn, multisequential_draw, site_seed
from ...layers.conformer import (ConvolutionModule, EncoderLayer, LayerNorm,
                                 PositionwiseFeedForward, RelPositionMultiHeadedAttention)
from ...layers.subsampling import Conv2dSubsampling, RelPositionalEncoding
from ... import hip_ops as ops
from ..._lib import lib


class TooShortUttError(Exception):
    """subsampling.py:14-28"""

    def __init__(self, message, actual_size, limit):
        super().__init__(message)
        self.actual_size = actual_size
        self.limit = limit


class AbsEncoder(nn.Module):
    def output_size(self) -> int:
        raise NotImplementedError


class _AfterNorm(nn.LayerNorm):
    def bind(self, arena, prefix, cd):
        from ...layers.common import Bound
        self._b = Bound(arena, prefix, cd)


class ConformerEncoder(AbsEncoder):
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
        input_layer: str = "conv2d",
        normalize_before: bool = True,
        concat_after: bool = False,
        positionwise_layer_type: str = "linear",
        positionwise_conv_kernel_size: int = 3,
        macaron_style: bool = False,
        rel_pos_type: str = "legacy",
        pos_enc_layer_type: str = "rel_pos",
        selfattention_layer_type: str = "rel_selfattn",
        activation_type: str = "swish",
        use_cnn_module: bool = True,
        zero_triu: bool = False,
        cnn_module_kernel: int = 31,
        padding_idx: int = -1,
        interctc_layer_idx: List[int] = [],
        interctc_use_conditioning: bool = False,
        stochastic_depth_rate: Union[float, List[float]] = 0.0,
        layer_drop_rate: float = 0.0,
        max_pos_emb_len: int = 5000,
    ):
        super().__init__()
        self._output_size = output_size
        # option resolution as conformer_encoder.py:117-143
        if rel_pos_type == "legacy":
            if pos_enc_layer_type == "rel_pos":
                pos_enc_layer_type = "legacy_rel_pos"
            if selfattention_layer_type == "rel_selfattn":
                selfattention_layer_type = "legacy_rel_selfattn"
        elif rel_pos_type == "latest":
            assert selfattention_layer_type != "legacy_rel_selfattn"
            assert pos_enc_layer_type != "legacy_rel_pos"
        else:
            raise ValueError("unknown rel_pos_type: " + rel_pos_type)
        if pos_enc_layer_type not in ("abs_pos", "scaled_abs_pos", "rel_pos", "legacy_rel_pos"):
            raise ValueError("unknown pos_enc_layer: " + pos_enc_layer_type)
        if selfattention_layer_type not in ("selfattn", "legacy_rel_selfattn", "rel_selfattn"):
            raise ValueError("unknown encoder_attn_layer: " + selfattention_layer_type)
        if input_layer not in ("linear", "conv2d", "conv2d1", "conv2d2", "conv2d6", "conv2d8",
                               "embed") and not isinstance(input_layer, nn.Module) and input_layer is not None:
            raise ValueError("unknown input_layer: " + str(input_layer))
        unsupported = []
        if pos_enc_layer_type != "rel_pos" or selfattention_layer_type != "rel_selfattn":
            unsupported.append(f"{pos_enc_layer_type}/{selfattention_layer_type}")
        if input_layer != "conv2d":
            unsupported.append(f"input_layer={input_layer}")
        if positionwise_layer_type != "linear":
            unsupported.append(f"positionwise_layer_type={positionwise_layer_type}")
        if activation_type != "swish":
            unsupported.append(f"activation_type={activation_type}")
        if interctc_layer_idx or stochastic_depth_rate not in (0, 0.0) or layer_drop_rate > 0:
            unsupported.append("interctc/stochastic depth/layer drop")
        if not normalize_before or concat_after or not use_cnn_module:
            unsupported.append("normalize_before=False/concat_after/use_cnn_module=False")
        if unsupported:
            raise NotImplementedError("espnet_amd ConformerEncoder implements the ASR recipes' "
                                      "configuration only; unsupported: " + ", ".join(unsupported))
        if output_size % 8:
            raise ValueError("output_size must be a multiple of 8 (16-B aligned MFMA operands)")
        self.embed = Conv2dSubsampling(input_size, output_size, dropout_rate,
                                       RelPositionalEncoding(output_size, positional_dropout_rate,
                                                             max_pos_emb_len))
        self.normalize_before = normalize_before
        layers = []
        for lnum in range(num_blocks):
            layers.append(EncoderLayer(
                output_size,
                RelPositionMultiHeadedAttention(attention_heads, output_size, attention_dropout_rate, zero_triu),
                PositionwiseFeedForward(output_size, linear_units, dropout_rate),
                PositionwiseFeedForward(output_size, linear_units, dropout_rate) if macaron_style else None,
                ConvolutionModule(output_size, cnn_module_kernel),
                dropout_rate, normalize_before, concat_after, 0.0))
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
            g += EncoderLayer.arena_groups(f"{prefix}encoders.{i}.")
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
        """conformer_encoder.py:300-377.  xs_pad (B,T,F) f32 on the GPU, ilens (B,) int64."""
        B, T, _ = xs_pad.shape
        if T < 7:  # check_short_utt, subsampling.py:31-43
            raise TooShortUttError(f"has {T} frames and is too short for subsampling "
                                   f"(it needs more than 7 frames), return empty results", T, 7)
        xs_pad = xs_pad.contiguous()
        olens = torch.empty(B, dtype=torch.long, device=xs_pad.device)
        lib.ea_subsample_lens(B, T, ilens.data_ptr(), olens.data_ptr(), ops.stream())
        x = self.embed(xs_pad, seed)
        multisequential_draw(len(self.encoders))
        T2 = x.shape[1]
        pos = self.embed.out[1].pos_emb(T2, x.device, self._cd, self.training, site_seed(seed, 0, 9))
        for layer in self.encoders:
            x = layer(x, pos, olens, seed)
        x = LayerNormFn.apply(x, self.after_norm)
        return x, olens, None
