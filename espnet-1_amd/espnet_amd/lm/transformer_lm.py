"""TransformerLM — drop-in for espnet2/lm/transformer_lm.py:12-130 as a decoding scorer (the
`scorers["lm"]` of espnet2/bin/asr_inference.py:149-183, LM shallow fusion in BeamSearch).

Same constructor, state_dict layout (embed, encoder.embed.{0,1}, encoder.encoders.{i}.*,
encoder.after_norm, decoder) and scorer interface (forward -> (logits, None), score,
batch_score -> next-token log-probabilities).  The HIP path: embedding lookup kernel, the
legacy Encoder's "linear" input layer (Linear GEMM -> LayerNorm eps 1e-5 -> ReLU,
transformer/encoder.py:120-127), TransformerEncoderLayer blocks with CAUSAL self-attention
(the fused attention kernels' causal mask = subsequent_mask, mask.py), after_norm, the output
Linear and the row log-softmax kernel.

MI355X layout: decoding recomputes the prefix on every step instead of the reference's
per-layer output cache (forward_one_step, encoder.py:353-379): prefixes are a few dozen tokens,
so one batched pass over all hypotheses' prefixes is a handful of launches, and the state is
None.  Inference only (train/eval forward without autograd); LM training, pos_enc
"sinusoidal" and padding tokens inside a prefix (token 0 before the end) raise.
"""
from __future__ import annotations

from typing import Any, List, Tuple

import torch
from torch import nn

from .. import hip_ops as ops
from .._lib import lib
from ..arena import ParamArena
from ..layers.common import LayerNormFn
from ..layers.conformer import MultiHeadedAttention, PositionwiseFeedForward
from ..layers.transformer import TransformerEncoderLayer
from ..asr.encoder.conformer_encoder import _AfterNorm


class _Encoder(nn.Module):
    """transformer/encoder.py Encoder(input_layer="linear", normalize_before=True) parameters."""

    def __init__(self, idim, attention_dim, attention_heads, linear_units, num_blocks, dropout_rate):
        super().__init__()
        self.embed = nn.Sequential(nn.Linear(idim, attention_dim), nn.LayerNorm(attention_dim),
                                   nn.Dropout(dropout_rate), nn.ReLU())
        layers = []
        for i in range(num_blocks):
            layers.append(TransformerEncoderLayer(
                attention_dim, MultiHeadedAttention(attention_heads, attention_dim, dropout_rate),
                PositionwiseFeedForward(attention_dim, linear_units, dropout_rate, activation="relu"),
                dropout_rate))
            layers[-1].layer_idx = 100 + i
            layers[-1].causal = True
        self.encoders = nn.Sequential(*layers)
        self.after_norm = _AfterNorm(attention_dim, eps=1e-12)


class TransformerLM(nn.Module):
    def __init__(self, vocab_size: int, pos_enc: str = None, embed_unit: int = 128, att_unit: int = 256,
                 head: int = 2, unit: int = 1024, layer: int = 4, dropout_rate: float = 0.5):
        super().__init__()
        if pos_enc not in (None, "sinusoidal"):
            raise ValueError(f"unknown pos-enc option: {pos_enc}")
        if pos_enc is not None:
            raise NotImplementedError("espnet_amd TransformerLM: pos_enc='sinusoidal' is not built")
        if att_unit % 8 or embed_unit % 8:
            raise ValueError("embed_unit and att_unit must be multiples of 8 (16-B aligned operands)")
        self.vocab_size = vocab_size
        self.embed = nn.Embedding(vocab_size, embed_unit)
        self.encoder = _Encoder(embed_unit, att_unit, head, unit, layer, dropout_rate)
        self.decoder = nn.Linear(att_unit, vocab_size)
        self.arena = None

    def arena_groups(self):
        g = []
        for i in range(len(self.encoder.encoders)):
            g += TransformerEncoderLayer.arena_groups(f"encoder.encoders.{i}.")
        return g

    def prepare(self, device="cuda", amp: bool = False):
        """Move the parameters into a flat arena on the GPU (amp: bf16 GEMM operands)."""
        device = torch.device(device)
        if device.type != "cuda":
            raise RuntimeError("espnet_amd runs on the GPU only (no CPU fallback)")
        cd = torch.bfloat16 if amp else torch.float32
        self.arena = ParamArena(self, device, self.arena_groups(), shadow_dtype=cd)
        for i, layer in enumerate(self.encoder.encoders):
            layer.bind(self.arena, f"encoder.encoders.{i}.", cd)
        self.encoder.after_norm.bind(self.arena, "encoder.after_norm.", cd)
        self._cd, self._device = cd, device
        if not self.__dict__.get("_hooked", False):
            self.register_load_state_dict_post_hook(lambda m, _: m.arena and m.arena.refresh_shadow())
            self.__dict__["_hooked"] = True
        return self

    def _w(self, name):
        return self.arena.view(name, which="shadow" if self._cd == torch.bfloat16 else "data")

    def _f(self, name):
        return self.arena.view(name)

    @torch.no_grad()
    def logits(self, ids: torch.Tensor) -> torch.Tensor:
        """(B, L) int64 token ids -> (B, L, vocab) f32 logits (transformer_lm.py:62-74)."""
        if self.arena is None:
            raise RuntimeError("TransformerLM.prepare(device) first")
        if torch.is_grad_enabled() and self.training:
            raise NotImplementedError("espnet_amd TransformerLM is a decoding scorer (no training)")
        dev, cd = self._device, self._cd
        ids = ids.to(dev, torch.int64).contiguous()
        B, L = ids.shape
        nz = ids != 0
        lens = nz.sum(-1)
        # ys_mask = ys != 0 (transformer_lm.py:56-60) as key lengths: padding only at the end
        if bool((nz.cumprod(-1).sum(-1) != lens).any()):
            raise NotImplementedError("token 0 inside a prefix (padding is only supported at the end)")
        N = B * L
        E = self.embed.embedding_dim
        d = self.decoder.in_features
        x0 = torch.empty(N, E, device=dev)
        zero_pe = torch.zeros(L, E, device=dev)
        lib.ea_embed_fwd(N, E, L, ids.data_ptr(), self._f("embed.weight").data_ptr(), 1.0, zero_pe.data_ptr(),
                         0.0, 0, x0.data_ptr(), ops.stream())
        h = torch.empty(N, d, device=dev)
        xin = x0 if cd == torch.float32 else x0.to(cd)
        ops.linear(xin, self._w("encoder.embed.0.weight"), h, epi=ops.make_epi(bias=self._f("encoder.embed.0.bias")))
        x = torch.empty(N, d, device=dev)
        mu, rs = torch.empty(N, device=dev), torch.empty(N, device=dev)
        ops.layernorm_fwd(h, self._f("encoder.embed.1.weight"), self._f("encoder.embed.1.bias"), x, mu, rs,
                          eps=1e-5)
        lib.ea_relu_f32_inplace(N * d, x.data_ptr(), ops.stream())
        x = x.view(B, L, d)
        for layer in self.encoder.encoders:
            x = layer(x, lens, 0)
        x = LayerNormFn.apply(x, self.encoder.after_norm)
        y = torch.empty(N, self.vocab_size, device=dev)
        xo = x.reshape(N, d)
        xo = xo if cd == torch.float32 else xo.to(cd)
        ops.linear(xo, self._w("decoder.weight"), y, epi=ops.make_epi(bias=self._f("decoder.bias")))
        return y.view(B, L, self.vocab_size)

    def forward(self, input: torch.Tensor, hidden: None = None) -> Tuple[torch.Tensor, None]:
        return self.logits(input), None

    def batch_score(self, ys: torch.Tensor, states: List[Any], xs: torch.Tensor) -> Tuple[torch.Tensor, List[Any]]:
        """transformer_lm.py:102-130: next-token log-probabilities of every prefix (n, vocab)."""
        lg = self.logits(ys)[:, -1].contiguous()
        out = torch.empty_like(lg)
        lib.ea_softmax_rows(lg.shape[0], lg.shape[1], lg.data_ptr(), lg.shape[1], out.data_ptr(), 1, ops.stream())
        return out, [None] * lg.shape[0]

    def score(self, y: torch.Tensor, state: Any, x: torch.Tensor) -> Tuple[torch.Tensor, Any]:
        """transformer_lm.py:76-100 for one prefix."""
        logp, st = self.batch_score(y.unsqueeze(0), [state], None)
        return logp[0], st[0]
