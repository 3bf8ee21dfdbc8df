"""TransformerDecoder — drop-in for espnet2/asr/decoder/transformer_decoder.py:232-281
(training forward :92-145).  Same constructor, state_dict keys and init order; the
forward is one HIP autograd node (layers/decoder.py: DecoderFn).

Inference (transformer_decoder.py:146-229: forward_one_step / score / batch_score): an
incremental decoder over a device key/value cache (DecoderKVCache) — each step computes only
the new position of every hypothesis: its self-attention keys/values are appended to the
cache, the encoder memory's cross-attention keys/values are projected once per memory (one
GEMM for all layers), and the next-token log-softmax is one row kernel (ea_softmax_rows).
The reference's cache holds each layer's outputs for the prefix and re-projects the prefix's
keys/values every step; the scores are the same (a causal decoder's prefix rows do not
depend on later tokens)."""
from __future__ import annotations

import math
import os
from typing import Tuple

import torch
from torch import nn

from ... import hip_ops as ops
from ..._lib import lib
from ...layers.common import (ACT_RELU, EPI_ACT, EPI_RESID, Bound, empty, ln_fwd, multisequential_draw)
from ...layers.conformer import LayerNorm, MultiHeadedAttention, PositionwiseFeedForward
from ...layers.decoder import (DecoderFn, DecoderLayer, PositionalEncoding, _kv_names, _mha_fwd,
                               decoder_arena_groups)


class DecoderKVCache:
    """Incremental-decoding state of n hypotheses after L prefix positions.

    kv: (num_blocks, n, L, 2d) in the compute dtype — every layer's self-attention [key |
    value] rows of every prefix position (one row per (hypothesis, position), so the new
    position's key/value projection is ONE GEMM writing both halves, and the attention reads
    keys at column 0 and values at column d with row stride 2d).  mem: the cross-attention
    keys/values of the encoder memory for all layers, (n*T, 2*d*num_blocks), with the memory
    lengths; shared by every step over that memory (MemoryKV)."""

    __slots__ = ("kv", "L", "mem")

    def __init__(self, kv, L, mem):
        self.kv, self.L, self.mem = kv, L, mem

    def select(self, rows):
        """The caches of hypotheses `rows` (device or host indices), in that order."""
        idx = torch.as_tensor(rows, dtype=torch.long, device=self.kv.device)
        return DecoderKVCache(self.kv.index_select(1, idx), self.L, self.mem)


class GraphStepKV:
    """Decoder state of n hypotheses inside a captured decoding run (DecodeGraphs): which of
    the run's two static key/value buffers holds positions [0, L), and the step it was
    written at (a state older than the previous step is stale: its buffer was reused)."""

    __slots__ = ("run", "n", "buf", "L", "step")

    def __init__(self, run, n, buf, L, step):
        self.run, self.n, self.buf, self.L, self.step = run, n, buf, L, step


class DecodeGraphs:
    """Captured incremental decoder steps over one encoder memory (inference, §8(f) row 4).

    Decoding is launch-bound: a step is ~80 small launches for ~10 hypotheses.  Here each
    hypothesis count n gets two hipGraphs of ONE step (one per direction between two static
    (num_blocks, n, Lcap, 2d) key/value buffers), captured once with static-shape inputs: the
    token ids and the position live in device buffers, the positional-encoding row is gathered
    by the position on the device, the new key/value row is written at the position with an
    index copy, and self-attention runs over Lcap keys masked to pos + 1 (the fused kernel
    stops at that length).  A step = one packed host->device copy, one row gather of the
    surviving hypotheses' caches (outside the graph: n may change between steps) and a replay."""

    def __init__(self, dec, memory: "MemoryKV", lcap: int):
        self.dec, self.mem, self.lcap = dec, memory, lcap
        self.per_n = {}
        self.nstep = 0  # steps run so far (a state from an older step is stale)

    def _setup(self, n):
        dec = self.dec
        b = dec._b
        dev = self.mem.memory.device
        nb = len(dec.decoders)
        d = dec.output_layer.in_features
        V = dec.output_layer.out_features
        st = dict(kv=[torch.zeros(nb, n, self.lcap, 2 * d, dtype=b.cd, device=dev) for _ in range(2)],
                  inp=torch.zeros(n + 1, dtype=torch.long, device=dev),   # [tokens | position]
                  host=torch.zeros(n + 1, dtype=torch.long).pin_memory(),
                  graphs=[None, None], out=[None, None], pool=None)
        self.per_n[n] = st
        dec._memory_kv(self.mem, n)  # cross-attention K/V before capture
        return st

    def _body(self, st, n, buf):
        """The step the graph captures: reads st['inp'], writes st['kv'][buf] row pos and the
        returned (n, V) log-probabilities."""
        dec = self.dec
        b = dec._b
        cd = b.cd
        nb = len(dec.decoders)
        d = dec.output_layer.in_features
        H = dec.decoders[0].self_attn.h
        dk = d // H
        V = dec.output_layer.out_features
        dev = st["inp"].device
        scale = 1.0 / math.sqrt(dk)
        mkv, hlens, Tm = dec._memory_kv(self.mem, n)
        ldm = 2 * d * nb
        tok = st["inp"][:n]
        pos = st["inp"][n:]
        kv = st["kv"][buf]
        klen = (pos + 1).expand(n).contiguous()
        pe = dec.embed[1]
        pe_row = pe.table(self.lcap, dev).index_select(0, pos)
        x = empty(n, d, device=dev)
        lib.ea_embed_fwd(n, d, 1, tok.data_ptr(), b.f("embed.0.weight").data_ptr(), pe.xscale, pe_row.data_ptr(),
                         0.0, 0, x.data_ptr(), ops.stream())
        # each LayerNorm computed inside the Linear that consumes it (ea_gemm_ln: few-row bf16)
        fuse_ln = cd == torch.bfloat16 and n <= 16 and d % 32 == 0 and d <= 2048

        def ln_linear(xin, norm, w, out, epi):
            if fuse_ln:
                return ops.linear_ln(xin, b.f(norm + ".weight"), b.f(norm + ".bias"), w, out, epi=epi)
            xn, _, _ = ln_fwd(xin, b, norm, cd)
            return ops.linear(xn, w, out, epi=epi)

        for l in range(nb):
            nm = f"decoders.{l}."
            sa, xa, ff = nm + "self_attn.", nm + "src_attn.", nm + "feed_forward."
            # q | k | v in one GEMM (adjacent in the arena); k | v of this position go to the cache
            qkv = empty(n, 3 * d, dtype=cd, device=dev)
            ln_linear(x, nm + "norm1", b.w(sa + "linear_q.weight", sa + "linear_k.weight", sa + "linear_v.weight",
                                           shape=(3 * d, d)), qkv,
                      ops.make_epi(bias=b.f(sa + "linear_q.bias", sa + "linear_k.bias", sa + "linear_v.bias",
                                            shape=(3 * d,))))
            kvl = kv[l]
            kvl.index_copy_(1, pos, qkv[:, d:].view(n, 1, 2 * d))
            O1, _ = _mha_fwd(qkv, kvl, kvl[:, :, d:], B=n, H=H, T1=1, T2=self.lcap, dk=dk, ldq=3 * d, ldk=2 * d,
                             ldv=2 * d, klen=klen, causal=False, scale=scale, p=0.0, seed=0, cd=cd)
            x1 = empty(n, d, device=dev)
            ops.linear(O1, b.w(sa + "linear_out.weight"), x1,
                       epi=ops.make_epi(EPI_RESID, bias=b.f(sa + "linear_out.bias"), resid=x))
            q2 = empty(n, d, dtype=cd, device=dev)
            ln_linear(x1, nm + "norm2", b.w(xa + "linear_q.weight"), q2, ops.make_epi(bias=b.f(xa + "linear_q.bias")))
            O2, _ = _mha_fwd(q2, mkv[:, 2 * d * l:], mkv[:, 2 * d * l + d:], B=n, H=H, T1=1, T2=Tm, dk=dk,
                             ldq=d, ldk=ldm, ldv=ldm, klen=hlens, causal=False, scale=scale, p=0.0, seed=0, cd=cd)
            x2 = empty(n, d, device=dev)
            ops.linear(O2, b.w(xa + "linear_out.weight"), x2,
                       epi=ops.make_epi(EPI_RESID, bias=b.f(xa + "linear_out.bias"), resid=x1))
            Fh = dec.decoders[l].feed_forward.w_1.out_features
            h = empty(n, Fh, dtype=cd, device=dev)
            a = empty(n, Fh, dtype=cd, device=dev)
            ln_linear(x2, nm + "norm3", b.w(ff + "w_1.weight"), a,
                      ops.make_epi(EPI_ACT, bias=b.f(ff + "w_1.bias"), act=ACT_RELU, aux=h))
            x3 = empty(n, d, device=dev)
            ops.linear(a, b.w(ff + "w_2.weight"), x3,
                       epi=ops.make_epi(EPI_RESID, bias=b.f(ff + "w_2.bias"), resid=x2))
            x = x3
        logits = empty(n, V, device=dev)
        ln_linear(x, "after_norm", b.w("output_layer.weight"), logits, ops.make_epi(bias=b.f("output_layer.bias")))
        logp = empty(n, V, device=dev)
        lib.ea_softmax_rows(n, V, logits.data_ptr(), V, logp.data_ptr(), 1, ops.stream())
        return logp

    def step(self, tok, pos, prev: "GraphStepKV", rows):
        """Score position pos (tok: host ints, n of them) for hypotheses whose caches are rows
        `rows` of prev (None at pos 0).  Returns (logp (n, V) — a static buffer, valid until
        the next step — and the new GraphStepKV)."""
        n = len(tok)
        st = self.per_n.get(n) or self._setup(n)
        buf = 0 if prev is None else 1 - prev.buf
        if prev is not None:
            # the surviving hypotheses' key/value rows of positions [0, pos) — the step writes
            # row pos and reads no further (klen = pos + 1)
            src = self.per_n[prev.n]["kv"][prev.buf]
            idx = torch.as_tensor(rows, dtype=torch.long).to(src.device, non_blocking=True)
            st["kv"][buf][:, :, :pos].copy_(torch.index_select(src[:, :, :pos], 1, idx))
        st["host"][:n] = torch.as_tensor(tok, dtype=torch.long)
        st["host"][n] = pos
        st["inp"].copy_(st["host"], non_blocking=True)
        if st["graphs"][buf] is None:
            self._body(st, n, buf)  # eager warm-up (lazy workspaces), then capture
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=st["pool"], capture_error_mode="thread_local"):
                st["out"][buf] = self._body(st, n, buf)
            st["pool"] = g.pool()
            st["graphs"][buf] = g
        st["graphs"][buf].replay()
        self.nstep += 1
        return st["out"][buf], GraphStepKV(self, n, buf, pos + 1, self.nstep)


class MemoryKV:
    """Cross-attention keys/values of one encoder memory for all decoder layers (the training
    forward's single K/V GEMM, layers/decoder.py), kept per hypothesis count n."""

    __slots__ = ("memory", "by_n")

    def __init__(self, memory):
        self.memory = memory
        self.by_n = {}


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
                         memory_mask=None, *, cache=None, return_hs=False):
        """transformer_decoder.py:146-184: log-softmax of the next token after each prefix in
        tgt (B, L) over memory (B, T, d) (no memory mask; tgt_mask is the causal mask the
        reference builds, implied here).  `cache`: the DecoderKVCache this method returned
        for tgt[:, :-1] (rows in tgt's order) — then only the last position is computed;
        None (or a cache of another length) builds it from the prefix first.  Returns
        (logp (B, V) f32, the cache of tgt)."""
        if memory_mask is not None:
            raise NotImplementedError("memory_mask is not used by the ASR scorers")
        B, L = tgt.shape
        dev = memory.device
        tgt = tgt.to(dev)
        if not isinstance(cache, DecoderKVCache) or cache.L != L - 1 or cache.kv.shape[1] != B:
            cache = self._empty_cache(memory)
            for pos in range(L - 1):  # prefill: the prefix one position at a time
                _, cache = self._step(tgt[:, pos], pos, cache)
        logp, hs, cache = self._step(tgt[:, -1], L - 1, cache, want_hs=True)
        if return_hs:
            return (logp, hs), cache
        return logp, cache

    def _empty_cache(self, memory):
        b = self._b
        B = memory.shape[0]
        d = memory.shape[2]
        kv = torch.empty(len(self.decoders), B, 0, 2 * d, dtype=b.cd, device=memory.device)
        return DecoderKVCache(kv, 0, MemoryKV(memory))

    def _memory_kv(self, mem: MemoryKV, n: int):
        """(n*T, 2*d*nb) cross-attention K/V rows and lengths of n hypotheses over the memory:
        one GEMM (all layers' src_attn.linear_k/linear_v are adjacent in the arena)."""
        got = mem.by_n.get(n)
        if got is not None:
            return got
        b = self._b
        m = mem.memory
        Bm, T, d = m.shape
        nb = len(self.decoders)
        if Bm == n:
            rows = m.reshape(n * T, d)
        elif Bm == 1 or m.stride(0) == 0:  # one memory shared by every hypothesis
            rows = m[:1].expand(n, T, d).reshape(n * T, d)
        else:
            raise ValueError(f"memory batch {Bm} does not match {n} hypotheses")
        kvw, kvb = _kv_names(nb)
        kv = empty(n * T, 2 * d * nb, dtype=b.cd, device=m.device)
        ops.linear(ops.cast(rows.contiguous(), b.cd), b.w(*kvw, shape=(2 * d * nb, d)), kv,
                   epi=ops.make_epi(bias=b.f(*kvb, shape=(2 * d * nb,))))
        hlens = torch.full((n,), T, dtype=torch.long, device=m.device)
        mem.by_n[n] = (kv, hlens, T)
        return mem.by_n[n]

    def _step(self, tok, pos, cache: DecoderKVCache, want_hs=False):
        """One position (index pos) for every hypothesis: tok (n,) the token at pos; cache
        holds positions [0, pos).  Returns (logp (n, V) f32, new cache) (+ the after_norm
        output when want_hs)."""
        b = self._b
        cd = b.cd
        nb = len(self.decoders)
        n = tok.shape[0]
        d = self.output_layer.in_features
        H = self.decoders[0].self_attn.h
        dk = d // H
        V = self.output_layer.out_features
        dev = tok.device
        scale = 1.0 / math.sqrt(dk)
        mkv, hlens, Tm = self._memory_kv(cache.mem, n)
        ldm = 2 * d * nb
        L1 = pos + 1
        kv = torch.empty(nb, n, L1, 2 * d, dtype=cd, device=dev)
        if pos:
            kv[:, :, :pos].copy_(cache.kv)
        klen = torch.full((n,), L1, dtype=torch.long, device=dev)
        pe = self.embed[1]
        x = empty(n, d, device=dev)
        tok = tok.reshape(n).to(torch.long).contiguous()
        table = pe.table(L1, dev)
        lib.ea_embed_fwd(n, d, 1, tok.data_ptr(), b.f("embed.0.weight").data_ptr(), pe.xscale,
                         table[pos:].data_ptr(), 0.0, 0, x.data_ptr(), ops.stream())
        for l in range(nb):
            nm = f"decoders.{l}."
            sa, xa, ff = nm + "self_attn.", nm + "src_attn.", nm + "feed_forward."
            xn1, _, _ = ln_fwd(x, b, nm + "norm1", cd)
            q = empty(n, d, dtype=cd, device=dev)
            ops.linear(xn1, b.w(sa + "linear_q.weight"), q, epi=ops.make_epi(bias=b.f(sa + "linear_q.bias")))
            kvl = kv[l]  # (n, L1, 2d): this position's [k | v] row written in place
            ops.linear(xn1, b.w(sa + "linear_k.weight", sa + "linear_v.weight", shape=(2 * d, d)), kvl[:, pos],
                       epi=ops.make_epi(bias=b.f(sa + "linear_k.bias", sa + "linear_v.bias", shape=(2 * d,))))
            O1, _ = _mha_fwd(q, kvl, kvl[:, :, d:], B=n, H=H, T1=1, T2=L1, dk=dk, ldq=d, ldk=2 * d, ldv=2 * d,
                             klen=klen, causal=False, scale=scale, p=0.0, seed=0, cd=cd)
            x1 = empty(n, d, device=dev)
            ops.linear(O1, b.w(sa + "linear_out.weight"), x1,
                       epi=ops.make_epi(EPI_RESID, bias=b.f(sa + "linear_out.bias"), resid=x))
            xn2, _, _ = ln_fwd(x1, b, nm + "norm2", cd)
            q2 = empty(n, d, dtype=cd, device=dev)
            ops.linear(xn2, b.w(xa + "linear_q.weight"), q2, epi=ops.make_epi(bias=b.f(xa + "linear_q.bias")))
            O2, _ = _mha_fwd(q2, mkv[:, 2 * d * l:], mkv[:, 2 * d * l + d:], B=n, H=H, T1=1, T2=Tm, dk=dk,
                             ldq=d, ldk=ldm, ldv=ldm, klen=hlens, causal=False, scale=scale, p=0.0, seed=0, cd=cd)
            x2 = empty(n, d, device=dev)
            ops.linear(O2, b.w(xa + "linear_out.weight"), x2,
                       epi=ops.make_epi(EPI_RESID, bias=b.f(xa + "linear_out.bias"), resid=x1))
            xn3, _, _ = ln_fwd(x2, b, nm + "norm3", cd)
            Fh = self.decoders[l].feed_forward.w_1.out_features
            h = empty(n, Fh, dtype=cd, device=dev)
            a = empty(n, Fh, dtype=cd, device=dev)
            ops.linear(xn3, b.w(ff + "w_1.weight"), a,
                       epi=ops.make_epi(EPI_ACT, bias=b.f(ff + "w_1.bias"), act=ACT_RELU, aux=h))
            x3 = empty(n, d, device=dev)
            ops.linear(a, b.w(ff + "w_2.weight"), x3,
                       epi=ops.make_epi(EPI_RESID, bias=b.f(ff + "w_2.bias"), resid=x2))
            x = x3
        xf, _, _ = ln_fwd(x, b, "after_norm", cd)
        logits = empty(n, V, device=dev)
        ops.linear(xf, b.w("output_layer.weight"), logits, epi=ops.make_epi(bias=b.f("output_layer.bias")))
        logp = empty(n, V, device=dev)
        lib.ea_softmax_rows(n, V, logits.data_ptr(), V, logp.data_ptr(), 1, ops.stream())
        new = DecoderKVCache(kv, L1, cache.mem)
        if want_hs:
            return logp, xf, new
        return logp, new

    @staticmethod
    def _as_cache(src):
        """A hypothesis state's cache as a DecoderKVCache: a GraphStepKV (a captured run's
        state, e.g. when a prefix outgrows graph_lcap or the memory changes) is viewed as its
        run's static buffer cropped to its L positions; a stale one (its buffer was reused by
        a later step) gives None, so the step re-builds the cache from the prefix."""
        if isinstance(src, GraphStepKV):
            run = src.run
            if src.step != run.nstep:
                return None
            kv = run.per_n[src.n]["kv"][src.buf][:, :, :src.L]
            return DecoderKVCache(kv, src.L, run.mem)
        return src

    def score(self, ys, state, x):
        """transformer_decoder.py:186-192 (one hypothesis); state = (DecoderKVCache, row)."""
        cache = None
        if isinstance(state, tuple):
            src = self._as_cache(state[0])
            cache = src.select([state[1]]) if src is not None else None
        logp, cache = self.forward_one_step(ys.unsqueeze(0), None, x.unsqueeze(0), cache=cache)
        return logp.squeeze(0), (cache, 0)

    # captured decoding steps (DecodeGraphs): on by default on the GPU; EA_DECODE_GRAPH=0 runs
    # the eager incremental step.  graph_lcap: key/value capacity (positions) of a captured run.
    decode_graph = os.environ.get("EA_DECODE_GRAPH", "1") != "0"
    graph_lcap = 512

    def _graph_batch_score(self, ys, states, xs):
        """batch_score on a captured run, or None when this call cannot use one (a prefix
        longer than the capacity, states of another run / a stale step, a new memory)."""
        n, L = ys.shape
        pos = L - 1
        if pos >= self.graph_lcap:
            return None
        prev, rows = None, None
        if pos > 0:
            if not (states and all(isinstance(s, tuple) and isinstance(s[0], GraphStepKV) for s in states)):
                return None
            prev = states[0][0]
            run = prev.run
            if any(s[0].run is not run or s[0].step != prev.step or s[0].L != pos for s in states) \
                    or prev.step != run.nstep or run.mem.memory.shape[1:] != xs.shape[1:]:
                return None
            rows = [s[1] for s in states]  # the parents' rows of the previous step's buffer
        else:
            mem = xs[:1] if (xs.shape[0] == 1 or xs.stride(0) == 0) else xs
            run = DecodeGraphs(self, MemoryKV(mem), self.graph_lcap)
        tok = ys[:, -1].tolist()
        logp, kv = run.step(tok, pos, prev, rows)
        return logp, [(kv, i) for i in range(n)]

    def batch_score(self, ys: torch.Tensor, states, xs: torch.Tensor):
        """transformer_decoder.py:194-229 (BatchScorerInterface): next-token scores of n
        prefixes (n, L) over xs (n, T, d).  A hypothesis's state is (cache, row) — its row of
        the batched key/value cache its parent was scored with; the step gathers the surviving
        rows once and computes only the new position (on a captured run, DecodeGraphs, when
        it can: a search that starts from the <sos> prefix)."""
        n = ys.shape[0]
        if self.decode_graph and not self.training and torch.cuda.is_available():
            got = self._graph_batch_score(ys, states, xs)
            if got is not None:
                return got
        cache = None
        if states and all(isinstance(s, tuple) for s in states):
            src = states[0][0]
            if all(s[0] is src for s in states) and src.L == ys.shape[1] - 1:
                src = self._as_cache(src)
                cache = src.select([s[1] for s in states]) if src is not None else None
                if cache is not None and cache.mem.memory.shape[1:] != xs.shape[1:]:
                    cache = None
        logp, new = self.forward_one_step(ys, None, xs, cache=cache)
        return logp, [(new, i) for i in range(n)]
