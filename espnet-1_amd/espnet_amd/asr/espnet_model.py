"""ESPnetASRModel — drop-in for espnet2/asr/espnet_model.py:37-338 (hybrid CTC/attention).

forward(speech, speech_lengths, text, text_lengths) -> (loss, stats, weight) with the
reference's semantics (text crop, sos/eos, loss = w*ctc + (1-w)*att, stats keys,
force_gatherable shapes).  Runtime: call `prepare(device, amp)` once after construction
(or after load_state_dict on CPU): it lays all parameters into the flat arena
(espnet_amd/arena.py) and binds every block to its HIP views.
"""
from __future__ import annotations

import ctypes
import logging
from typing import Dict, List, Optional, Tuple, Union

import torch
from torch import nn

from .. import hip_ops as ops
from .._lib import lib
from ..arena import ParamArena
from ..layers.common import site_seed
from ..layers.losses import CombineFn, LabelSmoothingLossFn
from .ctc import CTC
from .error_calculator import ErrorCalculator
from .abs_modules import AbsNormalize


class AbsESPnetModel(nn.Module):
    pass


class UtteranceMVN(AbsNormalize):
    """espnet2/layers/utterance_mvn.py:10-43 (norm_means=True, norm_vars=False)."""

    def __init__(self, norm_means: bool = True, norm_vars: bool = False, eps: float = 1.0e-20):
        super().__init__()
        if not norm_means or norm_vars:
            raise NotImplementedError("only norm_means=True, norm_vars=False (ASRTask default)")
        self.norm_means = norm_means
        self.norm_vars = norm_vars
        self.eps = eps

    def forward(self, x, ilens):
        B, T, F = x.shape
        y = torch.empty_like(x)
        n = ctypes.c_long(0)
        lib.ea_utterance_mvn_ws_bytes(B, T, F, ctypes.addressof(n))
        ws = torch.empty(max(n.value, 8), dtype=torch.uint8, device=x.device)
        lib.ea_utterance_mvn2(B, T, F, x.data_ptr(), ilens.data_ptr(), y.data_ptr(), ws.data_ptr(), ws.numel(),
                              ops.stream())
        return y, ilens


class LabelSmoothingLoss(nn.Module):
    """transformer/label_smoothing_loss.py:13-39 (KLDivLoss criterion)."""

    def __init__(self, size, padding_idx, smoothing, normalize_length=False):
        super().__init__()
        self.padding_idx = padding_idx
        self.confidence = 1.0 - smoothing
        self.smoothing = smoothing
        self.size = size
        self.normalize_length = normalize_length

    def forward(self, x, target):
        assert x.size(2) == self.size
        return LabelSmoothingLossFn.apply(x.contiguous(), target, self)


class ESPnetASRModel(AbsESPnetModel):
    def __init__(
        self,
        vocab_size: int,
        token_list: Union[Tuple[str, ...], List[str]],
        frontend=None,
        specaug=None,
        normalize=None,
        preencoder=None,
        encoder=None,
        postencoder=None,
        decoder=None,
        ctc: CTC = None,
        joint_network=None,
        aux_ctc: dict = None,
        ctc_weight: float = 0.5,
        interctc_weight: float = 0.0,
        ignore_id: int = -1,
        lsm_weight: float = 0.0,
        length_normalized_loss: bool = False,
        report_cer: bool = True,
        report_wer: bool = True,
        sym_space: str = "<space>",
        sym_blank: str = "<blank>",
        sym_sos: str = "<sos/eos>",
        sym_eos: str = "<sos/eos>",
        extract_feats_in_collect_stats: bool = True,
        lang_token_id: int = -1,
    ):
        assert 0.0 <= ctc_weight <= 1.0, ctc_weight
        assert 0.0 <= interctc_weight < 1.0, interctc_weight
        super().__init__()
        if preencoder is not None or postencoder is not None:
            raise NotImplementedError("preencoder/postencoder are outside the HIP hot path (SURVEY.md §2a)")
        if joint_network is not None or interctc_weight != 0.0 or lang_token_id != -1:
            raise NotImplementedError("transducer / interCTC / lang token are not on the path")
        self.blank_id = token_list.index(sym_blank) if sym_blank in token_list else 0
        self.sos = token_list.index(sym_sos) if sym_sos in token_list else vocab_size - 1
        self.eos = token_list.index(sym_eos) if sym_eos in token_list else vocab_size - 1
        if self.blank_id != 0:
            raise NotImplementedError("the CTC kernels use blank = 0 (torch CTCLoss default)")
        self.vocab_size = vocab_size
        self.ignore_id = ignore_id
        self.ctc_weight = ctc_weight
        self.interctc_weight = interctc_weight
        self.aux_ctc = aux_ctc
        self.token_list = list(token_list)
        self.frontend = frontend
        self.specaug = specaug
        self.normalize = normalize
        self.preencoder = None
        self.postencoder = None
        self.encoder = encoder
        self.encoder.interctc_use_conditioning = False
        self.use_transducer_decoder = False
        self.error_calculator = None
        if ctc_weight < 1.0:
            assert decoder is not None, "decoder should not be None when attention is used"
        else:
            decoder = None
            logging.warning("Set decoder to none as ctc_weight==1.0")
        self.decoder = decoder
        self.criterion_att = LabelSmoothingLoss(vocab_size, ignore_id, lsm_weight, length_normalized_loss)
        if report_cer or report_wer:  # espnet_model.py:164-167 (used in eval mode only)
            self.error_calculator = ErrorCalculator(token_list, sym_space, sym_blank, report_cer, report_wer)
        self.ctc = None if ctc_weight == 0.0 else ctc
        self.extract_feats_in_collect_stats = extract_feats_in_collect_stats
        self.is_encoder_whisper = False
        self.lang_token_id = None
        self.arena = None
        self.seed = 0
        self._step = 0
        # loading weights into a prepared model writes the f32 arena (the Parameters are its
        # views); under AMP the GEMMs read the bf16 shadow, so it is refreshed after every load
        # — of the whole model or of any submodule (model.encoder.load_state_dict, as the
        # reference's init_param / load_pretrained_model do; prepare() hooks every module).
        # torch runs the loaded module's pre-hook first and its post-hook last (after its
        # children's), so the shadow is refreshed once per load_state_dict call.  In-place
        # edits of parameters (e.g. under torch.no_grad()) are seen by no hook: call
        # arena.refresh_shadow() after them.
        self.__dict__["_load_root"] = None  # not a submodule attribute
        self.register_load_state_dict_pre_hook(self._load_pre_hook)
        self.register_load_state_dict_post_hook(self._load_post_hook)

    def _load_pre_hook(self, module, *args, **kwargs):
        if self.__dict__.get("_load_root") is None:
            self.__dict__["_load_root"] = module

    def _load_post_hook(self, module, incompatible_keys):
        if module is self.__dict__.get("_load_root"):
            self.__dict__["_load_root"] = None
            if self.arena is not None:
                self.arena.refresh_shadow()

    # ------------------------------------------------------------------ runtime
    def arena_groups(self):
        g = self.encoder.arena_groups("encoder.")
        if self.decoder is not None:
            g += self.decoder.arena_groups("decoder.")
        return g

    def prepare(self, device="cuda", amp: bool = False, seed: int = 0):
        """Move the model into the flat arena on `device`; amp=True runs GEMMs in bf16
        (trainer.py:41-50 autocast(bfloat16)), everything else (LayerNorm, softmax, BN,
        losses, optimizer, residual stream) stays f32."""
        device = torch.device(device)
        if device.type != "cuda":
            raise RuntimeError("espnet_amd runs on the GPU only (no CPU fallback)")
        if device.index is None:
            device = torch.device("cuda", torch.cuda.current_device())
        cd = torch.bfloat16 if amp else torch.float32
        for m in self.modules():
            for k, v in list(m._buffers.items()):
                if v is not None:
                    m._buffers[k] = v.to(device)
        self.arena = ParamArena(self, device, self.arena_groups(), shadow_dtype=cd)
        self.compute_dtype = cd
        if not self.__dict__.get("_sub_hooks", False):
            for m in self.modules():
                if m is not self:
                    m.register_load_state_dict_pre_hook(self._load_pre_hook)
                    m.register_load_state_dict_post_hook(self._load_post_hook)
            self.__dict__["_sub_hooks"] = True
        self._anchor = torch.zeros(1, device=device, requires_grad=True)
        self.encoder.bind(self.arena, "encoder.", cd, self._anchor)
        if self.decoder is not None:
            self.decoder.bind(self.arena, "decoder.", cd)
        if self.ctc is not None:
            self.ctc.bind(self.arena, "ctc.", cd)
        self.seed = seed
        self._device = device
        # per-step dropout salt in device memory (ea_set_rng_salt): advanced on the stream at
        # every training forward, so eager steps and hipGraph replays draw fresh masks alike
        self._rng_salt = torch.zeros(1, dtype=torch.int64, device=device)
        return self

    def __del__(self):
        # the library keeps a raw pointer to this model's salt buffer: drop it with the model
        token = getattr(self, "_salt_token", None)
        if token is None:  # prepared but never ran forward: the library never saw its salt
            return
        if ESPnetASRModel._salt_owner is token:
            try:
                lib.ea_set_rng_salt(None)
            except Exception:
                pass
            ESPnetASRModel._salt_owner = None

    _salt_owner = None

    def _next_seed(self):
        """Site seeds are fixed per (model seed, rank); the per-step variation of every
        dropout mask comes from the device salt, advanced here (on the stream)."""
        lib.ea_set_rng_salt(self._rng_salt.data_ptr())
        self._salt_token = object() if getattr(self, "_salt_token", None) is None else self._salt_token
        ESPnetASRModel._salt_owner = self._salt_token
        if self.training:
            self._step += 1
            lib.ea_rng_advance(self._rng_salt.data_ptr(), ops.stream())
        rank = torch.distributed.get_rank() if torch.distributed.is_initialized() else 0
        return site_seed(self.seed + 1, 0, 1000 + rank)

    def _dev(self, t, dtype=None):
        if t.device != self._device:
            t = t.to(self._device, non_blocking=True)
        if dtype is not None and t.dtype != dtype:
            t = t.to(dtype)
        return t

    # ------------------------------------------------------------------ reference API
    def forward(self, speech: torch.Tensor, speech_lengths: torch.Tensor, text: torch.Tensor,
                text_lengths: torch.Tensor, **kwargs) -> Tuple[torch.Tensor, Dict[str, torch.Tensor], torch.Tensor]:
        assert text_lengths.dim() == 1, text_lengths.shape
        assert speech.shape[0] == speech_lengths.shape[0] == text.shape[0] == text_lengths.shape[0], \
            (speech.shape, speech_lengths.shape, text.shape, text_lengths.shape)
        batch_size = speech.shape[0]
        seed = self._next_seed()
        # host-side maxima (the reference syncs here too: text_lengths.max(), :218/:420);
        # a captured step (train/graph.py) passes them in, its lengths live on the device
        maxlens = kwargs.get("_maxlens")
        if maxlens is not None:
            sl_max, tl_max = maxlens
        else:
            tl_max = int(text_lengths.max())
            sl_max = int(speech_lengths.max())
        text = self._dev(text)[:, :tl_max]
        if self.ignore_id != -1:
            text = text.masked_fill(text == -1, self.ignore_id)
        text_lengths = self._dev(text_lengths, torch.long)
        encoder_out, encoder_out_lens = self.encode(speech, speech_lengths, _seed=seed, _smax=sl_max,
                                                    _lens_host=kwargs.get("_lens_host"))
        self._last_encoder_out = (encoder_out, encoder_out_lens)
        stats = dict()
        loss_ctc = loss_att = acc_att = None
        if self.ctc_weight != 0.0:
            loss_ctc = self.ctc(encoder_out, encoder_out_lens, text.contiguous(), text_lengths,
                                seed=site_seed(seed, 500, 1), overlap=True)
            stats["loss_ctc"] = loss_ctc.detach()
            stats["cer_ctc"] = None
            if not self.training and self.error_calculator is not None:  # :571-575
                ys_hat = self.ctc.argmax(encoder_out)
                stats["cer_ctc"] = self.error_calculator(ys_hat.cpu(), text.cpu(), is_ctc=True)
        if self.ctc_weight != 1.0:
            loss_att, acc_att = self._calc_att_loss(encoder_out, encoder_out_lens, text, text_lengths,
                                                    seed=site_seed(seed, 600, 1))
            stats["loss_att"] = loss_att.detach()
            stats["acc"] = acc_att
            stats["cer"] = None
            stats["wer"] = None
            if not self.training and self.error_calculator is not None:  # :551-557
                stats["cer"], stats["wer"] = self.error_calculator(self._att_argmax(), text.cpu())
        else:
            stats["loss_att"] = None
            stats["acc"] = None
            stats["cer"] = None
            stats["wer"] = None
        ops.join_aux()  # the CTC lattice ran on the auxiliary stream beside the decoder
        if self.ctc_weight == 0.0:
            loss = loss_att
        elif self.ctc_weight == 1.0:
            loss = loss_ctc
        else:
            ops.take_aux_fork()  # drop a fork point left by an earlier backward, if any
            loss = CombineFn.apply(loss_ctc, loss_att, float(self.ctc_weight))
        stats["loss"] = loss.detach()
        # force_gatherable (device_funcs.py:36-71): 0-d -> (1,), int weight -> int64 tensor
        stats = {k: (v.view(1) if isinstance(v, torch.Tensor)
                     else torch.tensor([v], dtype=torch.float, device=loss.device) if isinstance(v, float)
                     else v) for k, v in stats.items()}
        weight = torch.full((1,), batch_size, dtype=torch.long, device=loss.device)
        return loss.view(1), stats, weight

    def collect_feats(self, speech, speech_lengths, text, text_lengths, **kwargs):
        feats, feats_lengths = self._extract_feats(speech, speech_lengths)
        return {"feats": feats, "feats_lengths": feats_lengths}

    def _extract_feats(self, speech, speech_lengths, smax=None):
        """espnet_model.py:414-431: crop to the longest utterance, then the frontend (raw
        waveform -> log-mel frames) when there is one."""
        smax = int(speech_lengths.max()) if smax is None else smax
        speech, lens = self._dev(speech)[:, :smax], self._dev(speech_lengths, torch.long)
        if self.frontend is not None:
            return self.frontend(speech, lens)
        return speech, lens

    def encode(self, speech, speech_lengths, _seed=None, _smax=None, _lens_host=None):
        """espnet_model.py:351-412 (feats -> specaug (training) -> normalize -> encoder).
        `_lens_host`: the lengths as host ints, when the caller has them (SpecAug's
        equal-length test needs them on the host, time_warp.py:73)."""
        seed = self._next_seed() if _seed is None else _seed
        if self.specaug is not None and self.training and _lens_host is None and speech_lengths.device.type == "cpu":
            _lens_host = [int(v) for v in speech_lengths.tolist()]
        feats, feats_lengths = self._extract_feats(speech, speech_lengths, _smax)
        if self.frontend is not None and _lens_host is not None:  # sample counts -> frame counts
            _lens_host = [int(self.frontend.stft.frames_lens(int(v))) for v in _lens_host]
        feats = feats.contiguous().float()
        if self.specaug is not None and self.training:  # :365-366
            feats, feats_lengths = self.specaug(feats, feats_lengths, lens_host=_lens_host)
        if self.normalize is not None:
            feats, feats_lengths = self.normalize(feats, feats_lengths)
        encoder_out, encoder_out_lens, _ = self.encoder(feats, feats_lengths, seed=seed)
        return encoder_out, encoder_out_lens

    def _att_argmax(self):
        """decoder_out.argmax(dim=-1) (espnet_model.py:555) on the device, first maximal index."""
        lg = self._last_decoder_out.float().contiguous()
        B, L1, V = lg.shape
        out = torch.empty(B, L1, dtype=torch.long, device=lg.device)
        lib.ea_argmax_rows(B * L1, V, lg.data_ptr(), V, out.data_ptr(), ops.stream())
        return out.cpu()

    def _calc_att_loss(self, encoder_out, encoder_out_lens, ys_pad, ys_pad_lens, seed=0):
        """espnet_model.py:518-553 (training path: cer/wer None)."""
        B, L = ys_pad.shape
        ys_pad = ys_pad.contiguous()
        ys_in = torch.empty(B, L + 1, dtype=torch.long, device=ys_pad.device)
        ys_out = torch.empty(B, L + 1, dtype=torch.long, device=ys_pad.device)
        ys_in_lens = torch.empty(B, dtype=torch.long, device=ys_pad.device)
        lib.ea_add_sos_eos(B, L, ys_pad.data_ptr(), ys_pad.stride(0), ys_pad_lens.data_ptr(), self.sos,
                           self.eos, self.ignore_id, ys_in.data_ptr(), ys_out.data_ptr(),
                           ys_in_lens.data_ptr(), ops.stream())
        decoder_out, _ = self.decoder(encoder_out, encoder_out_lens, ys_in, ys_in_lens, seed=seed)
        loss_att, acc_att = self.criterion_att(decoder_out, ys_out)
        self._last_decoder_out = decoder_out
        return loss_att, acc_att
