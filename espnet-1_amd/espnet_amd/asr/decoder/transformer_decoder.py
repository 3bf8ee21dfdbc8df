"""TransformerDecoder — drop-in for espnet2/asr/decoder/transformer_decoder.py:232-281
(training forward :92-145).  Same constructor, state_dict keys and init order; the
forward is one HIP autograd node (layers/decoder.py: DecoderFn)."""
from __future__ import annotations

from typing import Tuple

import torch
from torch import nn

from ...layers.common import Bound, multisequential_draw
from ...layers.conformer import LayerNorm, MultiHeadedAttention, PositionwiseFeedForward
from ...layers.decoder import DecoderFn, DecoderLayer, PositionalEncoding, decoder_arena_groups


class AbsDecoder(nn.Module):
    pass


class TransformerDecoder(AbsDecoder):
    def __init__(
        self,
        vocab_size: int,
        encoder_output_size: int,
        attention_heads: int = 4,
        linear_units: int = 2048,
        num_blocks: int = 6,
        dropout_rate: float = 0.1,
        positional_dropout_rate: float = 0.1,
        self_attention_dropout_rate: float = 0.0,
        src_attention_dropout_rate: float = 0.0,
        input_layer: str = "embed",
        use_output_layer: bool = True,
        pos_enc_class=PositionalEncoding,
        normalize_before: bool = True,
        concat_after: bool = False,
        layer_drop_rate: float = 0.0,
    ):
        super().__init__()
        if input_layer != "embed":
            raise NotImplementedError("only input_layer='embed' (the ASR recipes) is implemented")
        if not use_output_layer or not normalize_before or concat_after or layer_drop_rate > 0:
            raise NotImplementedError("only use_output_layer/normalize_before=True, concat_after=False")
        attention_dim = encoder_output_size
        # BaseTransformerDecoder.__init__ order (transformer_decoder.py:64-86)
        self.embed = nn.Sequential(nn.Embedding(vocab_size, attention_dim),
                                   PositionalEncoding(attention_dim, positional_dropout_rate))
        self.normalize_before = normalize_before
        self.after_norm = LayerNorm(attention_dim)
        self.output_layer = nn.Linear(attention_dim, vocab_size)
        self.decoders = nn.Sequential(*[
            DecoderLayer(attention_dim,
                         MultiHeadedAttention(attention_heads, attention_dim, self_attention_dropout_rate),
                         MultiHeadedAttention(attention_heads, attention_dim, src_attention_dropout_rate),
                         PositionwiseFeedForward(attention_dim, linear_units, dropout_rate, "relu"),
                         dropout_rate, normalize_before, concat_after)
            for _ in range(num_blocks)])
        self.dropout_rate = dropout_rate
        self.self_attention_dropout_rate = self_attention_dropout_rate
        self.src_attention_dropout_rate = src_attention_dropout_rate
        self._b = None

    def arena_groups(self, prefix=""):
        return decoder_arena_groups(prefix, len(self.decoders))

    def bind(self, arena, prefix, cd):
        self._b = Bound(arena, prefix, cd)

    def forward(self, hs_pad: torch.Tensor, hlens: torch.Tensor, ys_in_pad: torch.Tensor,
                ys_in_lens: torch.Tensor, seed: int = 0) -> Tuple[torch.Tensor, torch.Tensor]:
        multisequential_draw(len(self.decoders))
        x = DecoderFn.apply(hs_pad.contiguous(), hlens, ys_in_pad.contiguous(), ys_in_lens, self,
                            seed, self.training)
        return x, ys_in_lens

    # ------------------------------------------------------------------ inference scorer
    @torch.no_grad()
    def forward_one_step(self, tgt: torch.Tensor, tgt_mask: torch.Tensor, memory: torch.Tensor,
                         cache=None):
        """transformer_decoder.py:146-184: log-softmax of the next token after each prefix
        in tgt (B, L) over memory (B, T, d), no memory mask.  The prefix is recomputed with
        the fused kernels instead of extending per-layer caches (a causal decoder's prefix
        outputs do not depend on later tokens, so the scores are the reference's); the
        returned `cache` is the per-layer placeholder list the reference's API passes on."""
        B, L = tgt.shape
        dev = memory.device
        hlens = torch.full((B,), memory.shape[1], dtype=torch.long, device=dev)
        ylens = torch.full((B,), L, dtype=torch.long, device=dev)
        logits = DecoderFn.apply(memory.contiguous(), hlens, tgt.to(dev).contiguous(), ylens, self, 0, False)
        y = torch.log_softmax(logits[:, -1].float(), dim=-1)
        return y, [None] * len(self.decoders)

    def score(self, ys, state, x):
        """transformer_decoder.py:186-192 (one hypothesis)."""
        logp, state = self.forward_one_step(ys.unsqueeze(0), None, x.unsqueeze(0), cache=state)
        return logp.squeeze(0), state

    def batch_score(self, ys: torch.Tensor, states, xs: torch.Tensor):
        """transformer_decoder.py:194-229: scores of the next token for a batch of prefixes."""
        logp, st = self.forward_one_step(ys, None, xs, cache=None)
        return logp, [[None] * len(self.decoders) for _ in range(len(ys))]
