"""espnet_amd — MI355X-native ESPnet2 ASR training step (hand-written HIP for gfx950).

Drop-in for the reference's ESPnetASRModel training path: same YAML keys,
same state_dict layout, same forward/backward semantics; every op runs in
libespnet_amd.so (see include/espnet_amd.h).
"""
__version__ = "0.1.0"

import os as _os

# The training step is captured as a hipGraph WITH its RCCL collectives.  ProcessGroupNCCL
# recycles CUDA events between work objects by default; an event recycled into a captured
# collective, while the process-group watchdog still polls the eager warm-up step's work that
# owned it, makes the watchdog's query fail ("event last recorded in a capturing stream") and
# abort the process.  Fresh events per work object keep the two apart.  Must be set before the
# process group is created (read at construction).
_os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")

