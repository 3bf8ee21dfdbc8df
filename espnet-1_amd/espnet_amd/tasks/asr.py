"""ASRTask — mirrors espnet2/tasks/asr.py: the class-choice registries (:88-188, with
their type checks), the task options (add_task_arguments :216-355), the collate / data
names (:357-440) and build_model (:476-602).

    python -m espnet_amd.bin.asr_train --config conf/train_asr_conformer8.yaml \
        --train_data_path_and_name_and_type dump/train/feats.scp,speech,npy ...

`build_model(args)` accepts the reference's YAML/argparse keys (input_size, token_list,
encoder/encoder_conf, decoder/decoder_conf, ctc_conf, model_conf, normalize/normalize_conf,
specaug/specaug_conf, frontend/frontend_conf) as a dict or a Namespace and builds the
HIP-backed modules; names outside the hot path raise with the reference's ValueError or a
NotImplementedError naming the reason.
"""
from __future__ import annotations

import argparse
import logging
from typing import Tuple

import numpy as np

from ..asr.abs_modules import AbsFrontend, AbsNormalize, AbsSpecAug
from ..asr.ctc import CTC
from ..asr.decoder.transformer_decoder import AbsDecoder, TransformerDecoder
from ..asr.encoder.conformer_encoder import AbsEncoder, ConformerEncoder
from ..asr.encoder.transformer_encoder import TransformerEncoder
from ..asr.espnet_model import AbsESPnetModel, ESPnetASRModel, UtteranceMVN
from ..asr.frontend.default import DefaultFrontend, GlobalMVN
from ..asr.specaug import SpecAug
from ..train.class_choices import ClassChoices
from ..train.collate_fn import CommonCollateFn
from ..utils.nested_dict_action import NestedDictAction
from ..utils.types import float_or_none, int_or_none, str2bool, str_or_none
from .abs_task import AbsTask, _default_kwargs

frontend_choices = ClassChoices("frontend", dict(default=DefaultFrontend), type_check=AbsFrontend,
                                default="default")
specaug_choices = ClassChoices("specaug", dict(specaug=SpecAug), type_check=AbsSpecAug, default=None, optional=True)
normalize_choices = ClassChoices("normalize", dict(global_mvn=GlobalMVN, utterance_mvn=UtteranceMVN),
                                 type_check=AbsNormalize, default="utterance_mvn", optional=True)
model_choices = ClassChoices("model", dict(espnet=ESPnetASRModel), type_check=AbsESPnetModel, default="espnet")
encoder_choices = ClassChoices("encoder", dict(conformer=ConformerEncoder, transformer=TransformerEncoder),
                               type_check=AbsEncoder, default="rnn")
decoder_choices = ClassChoices("decoder", dict(transformer=TransformerDecoder), type_check=AbsDecoder, default=None,
                               optional=True)
# the registries the reference also exposes, empty here (nothing on the training path uses them)
preencoder_choices = ClassChoices("preencoder", dict(), default=None, optional=True)
postencoder_choices = ClassChoices("postencoder", dict(), default=None, optional=True)


class _IntTextPreprocessor:
    """The part of CommonPreprocessor (espnet2/train/preprocessor.py:323-329) the ASR path
    needs: integer token sequences pass through unchanged; "char" tokenisation of string
    text uses the token list (spaces -> "<space>", unknown -> "<unk>").  Other token
    types need a tokenizer model (sentencepiece, g2p, ...) and raise."""

    def __init__(self, token_type, token_list):
        self.token_type = token_type
        self.token_list = list(token_list) if token_list is not None else None
        self.tok2id = {t: i for i, t in enumerate(self.token_list or [])}

    def __call__(self, uid, data):
        text = data.get("text")
        if text is None or isinstance(text, np.ndarray):
            return data
        if self.token_type != "char" or self.token_list is None:
            raise NotImplementedError(f"text tokenisation with token_type={self.token_type} (give integer "
                                      "token sequences, e.g. a text_int file, or --token_type char)")
        unk = self.tok2id.get("<unk>")
        ids = [self.tok2id.get("<space>" if c == " " else c, unk) for c in str(text)]
        data["text"] = np.array(ids, dtype=np.int64)
        return data


class ASRTask(AbsTask):
    num_optimizers: int = 1
    class_choices_list = [frontend_choices, specaug_choices, normalize_choices, model_choices, preencoder_choices,
                          encoder_choices, postencoder_choices, decoder_choices]

    @classmethod
    def add_task_arguments(cls, parser: argparse.ArgumentParser):
        g = parser.add_argument_group(description="Task related")
        required = parser.get_default("required")
        required += ["token_list"]
        g.add_argument("--token_list", type=str_or_none, default=None, help="A text mapping int-id to token")
        g.add_argument("--init", type=lambda x: str_or_none(x.lower()), default=None,
                       choices=["chainer", "xavier_uniform", "xavier_normal", "kaiming_uniform", "kaiming_normal",
                                None], help="The initialization method")
        g.add_argument("--input_size", type=int_or_none, default=None,
                       help="The number of input dimension of the feature")
        g.add_argument("--ctc_conf", action=NestedDictAction, default=_default_kwargs(CTC),
                       help="The keyword arguments for CTC class.")
        g.add_argument("--joint_net_conf", action=NestedDictAction, default=None,
                       help="The keyword arguments for joint network class.")
        g = parser.add_argument_group(description="Preprocess related")
        g.add_argument("--use_preprocessor", type=str2bool, default=True)
        g.add_argument("--token_type", type=str, default="bpe",
                       choices=["bpe", "char", "word", "phn", "hugging_face", "whisper_en", "whisper_multilingual"])
        g.add_argument("--bpemodel", type=str_or_none, default=None)
        parser.add_argument("--non_linguistic_symbols", type=str_or_none)
        g.add_argument("--cleaner", type=str_or_none, default=None,
                       choices=[None, "tacotron", "jaconv", "vietnamese", "whisper_en", "whisper_basic"])
        g.add_argument("--g2p", type=str_or_none, default=None)
        g.add_argument("--speech_volume_normalize", type=float_or_none, default=None)
        g.add_argument("--rir_scp", type=str_or_none, default=None)
        g.add_argument("--rir_apply_prob", type=float, default=1.0)
        g.add_argument("--noise_scp", type=str_or_none, default=None)
        g.add_argument("--noise_apply_prob", type=float, default=1.0)
        g.add_argument("--noise_db_range", type=str, default="13_15")
        g.add_argument("--short_noise_thres", type=float, default=0.5)
        g.add_argument("--aux_ctc_tasks", type=str, nargs="+", default=[])
        for cc in cls.class_choices_list:
            cc.add_arguments(g)
        g.add_argument("--preprocessor", type=lambda x: str_or_none(x.lower()), default="default",
                       choices=["default", "multi"], help="The preprocessor type")
        g.add_argument("--preprocessor_conf", action=NestedDictAction, default=dict())

    @classmethod
    def build_collate_fn(cls, args, train: bool):
        return CommonCollateFn(float_pad_value=0.0, int_pad_value=-1)  # asr.py:398 (0 is the CTC blank)

    @classmethod
    def build_preprocess_fn(cls, args, train: bool):
        if not getattr(args, "use_preprocessor", False):
            return None
        for key in ("rir_scp", "noise_scp", "speech_volume_normalize", "non_linguistic_symbols", "cleaner", "g2p"):
            if getattr(args, key, None) is not None:
                raise NotImplementedError(f"--{key}: the build's data path feeds features and integer text only")
        token_list = args.token_list
        if isinstance(token_list, str):
            with open(token_list, encoding="utf-8") as f:
                token_list = [line.rstrip() for line in f]
        return _IntTextPreprocessor(args.token_type, token_list)

    @classmethod
    def required_data_names(cls, train: bool = True, inference: bool = False) -> Tuple[str, ...]:
        return ("speech", "text") if not inference else ("speech",)

    @classmethod
    def optional_data_names(cls, train: bool = True, inference: bool = False) -> Tuple[str, ...]:
        return tuple(f"text_spk{n}" for n in range(2, 5))

    @classmethod
    def build_model(cls, args) -> ESPnetASRModel:
        return build_model(args)


def _get(args, key, default=None):
    if isinstance(args, dict):
        return args.get(key, default)
    return getattr(args, key, default)


def build_model(args) -> ESPnetASRModel:
    """asr.py:476-602."""
    token_list = _get(args, "token_list")
    if isinstance(token_list, str):
        with open(token_list, encoding="utf-8") as f:
            token_list = [line.rstrip() for line in f]
        if isinstance(args, argparse.Namespace):
            args.token_list = list(token_list)  # asr.py:483-489: overwrite the path with the list
    token_list = list(token_list)
    vocab_size = len(token_list)
    logging.info(f"Vocabulary size: {vocab_size}")
    if _get(args, "init") is not None:
        raise NotImplementedError(f"--init {_get(args, 'init')}: the recipes use torch's default initialisation")
    input_size = _get(args, "input_size")
    frontend = None
    if input_size is None:  # asr.py:491-501: raw waveform -> frontend -> features
        fe_cls = frontend_choices.get_class(_get(args, "frontend") or "default")
        frontend = fe_cls(**(_get(args, "frontend_conf") or {}))
        input_size = frontend.output_size()
    spec_cls = specaug_choices.get_class(_get(args, "specaug"))
    specaug = spec_cls(**(_get(args, "specaug_conf") or {})) if spec_cls else None
    norm_cls = normalize_choices.get_class(_get(args, "normalize", "utterance_mvn"))
    normalize = norm_cls(**(_get(args, "normalize_conf") or {})) if norm_cls else None
    for opt in ("preencoder", "postencoder"):
        if _get(args, opt) is not None:
            raise NotImplementedError(f"--{opt} is outside the HIP hot path (SURVEY.md §2a)")
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
