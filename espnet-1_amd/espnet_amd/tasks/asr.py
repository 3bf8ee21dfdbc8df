"""ASRTask model builder — mirrors espnet2/tasks/asr.py:476-602 (build_model) and the
class-choice registries of :109-188 for the names on the hot path.

`build_model(args)` accepts the reference's YAML/argparse keys (input_size, token_list,
encoder/encoder_conf, decoder/decoder_conf, ctc_conf, model_conf, normalize/normalize_conf,
specaug/specaug_conf, frontend/frontend_conf) and builds the HIP-backed modules; names outside the hot path raise
NotImplementedError with the reason.
"""
from __future__ import annotations

import argparse
from typing import Any, Dict

from ..asr.ctc import CTC
from ..asr.decoder.transformer_decoder import TransformerDecoder
from ..asr.encoder.conformer_encoder import AbsEncoder, ConformerEncoder
from ..asr.encoder.transformer_encoder import TransformerEncoder
from ..asr.espnet_model import ESPnetASRModel, UtteranceMVN
from ..asr.frontend.default import DefaultFrontend, GlobalMVN
from ..asr.specaug import SpecAug


class ClassChoices:
    """espnet2/train/class_choices.py:9-92 (lower-cased name -> class)."""

    def __init__(self, name, classes: Dict[str, type], default=None, optional=False):
        self.name = name
        self.classes = {k.lower(): v for k, v in classes.items()}
        self.default = default
        self.optional = optional

    def choices(self):
        return list(self.classes) + (["none", None] if self.optional else [])

    def get_class(self, name):
        if name is None or (self.optional and str(name).lower() == "none"):
            return None
        key = str(name).lower()
        if key not in self.classes:
            raise ValueError(f"--{self.name} must be one of {self.choices()}: --{self.name} {name}")
        return self.classes[key]


encoder_choices = ClassChoices("encoder", dict(conformer=ConformerEncoder, transformer=TransformerEncoder),
                                default="rnn")
decoder_choices = ClassChoices("decoder", dict(transformer=TransformerDecoder), default=None,
                               optional=True)
normalize_choices = ClassChoices("normalize", dict(utterance_mvn=UtteranceMVN, global_mvn=GlobalMVN),
                                 default="utterance_mvn", optional=True)
frontend_choices = ClassChoices("frontend", dict(default=DefaultFrontend), default="default")
model_choices = ClassChoices("model", dict(espnet=ESPnetASRModel), default="espnet")
specaug_choices = ClassChoices("specaug", dict(specaug=SpecAug), default=None, optional=True)


def _get(args, key, default=None):
    if isinstance(args, dict):
        return args.get(key, default)
    return getattr(args, key, default)


def build_model(args) -> ESPnetASRModel:
    token_list = _get(args, "token_list")
    if isinstance(token_list, str):
        with open(token_list, encoding="utf-8") as f:
            token_list = [line.rstrip() for line in f]
    token_list = list(token_list)
    vocab_size = len(token_list)
    input_size = _get(args, "input_size")
    frontend = None
    if input_size is None:  # tasks/asr.py:491-501: raw waveform -> frontend -> features
        fe_cls = frontend_choices.get_class(_get(args, "frontend") or "default")
        frontend = fe_cls(**(_get(args, "frontend_conf") or {}))
        input_size = frontend.output_size()
    spec_cls = specaug_choices.get_class(_get(args, "specaug"))
    specaug = spec_cls(**(_get(args, "specaug_conf") or {})) if spec_cls else None
    norm_cls = normalize_choices.get_class(_get(args, "normalize", "utterance_mvn"))
    normalize = norm_cls(**(_get(args, "normalize_conf") or {})) if norm_cls else None
    enc_cls = encoder_choices.get_class(_get(args, "encoder", "conformer"))
    encoder = enc_cls(input_size=input_size, **(_get(args, "encoder_conf") or {}))
    dec_cls = decoder_choices.get_class(_get(args, "decoder"))
    decoder = None
    if dec_cls is not None:
        decoder = dec_cls(vocab_size=vocab_size, encoder_output_size=encoder.output_size(),
                          **(_get(args, "decoder_conf") or {}))
    ctc = CTC(odim=vocab_size, encoder_output_size=encoder.output_size(), **(_get(args, "ctc_conf") or {}))
    model_cls = model_choices.get_class(_get(args, "model", "espnet") or "espnet")
    return model_cls(vocab_size=vocab_size, frontend=frontend, specaug=specaug, normalize=normalize,
                     preencoder=None, encoder=encoder, postencoder=None, decoder=decoder, ctc=ctc,
                     joint_network=None, token_list=token_list, **(_get(args, "model_conf") or {}))
