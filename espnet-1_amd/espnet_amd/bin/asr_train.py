"""python -m espnet_amd.bin.asr_train — espnet2/bin/asr_train.py:10-19 (ASRTask.main)."""
from __future__ import annotations

from ..tasks.asr import ASRTask


def get_parser():
    return ASRTask.get_parser()


def main(cmd=None):
    ASRTask.main(cmd=cmd)


if __name__ == "__main__":
    main()
