"""espnet_amd — MI355X-native ESPnet2 ASR training step (hand-written HIP for gfx950).

Drop-in for the reference's ESPnetASRModel training path: same YAML keys,
same state_dict layout, same forward/backward semantics; every op runs in
libespnet_amd.so (see include/espnet_amd.h).
"""
__version__ = "0.1.0"

# TORCH_NCCL_CUDA_EVENT_CACHE=0 is set where this package creates an RCCL process group
# (train.graph.prepare_nccl_env), not on import.
