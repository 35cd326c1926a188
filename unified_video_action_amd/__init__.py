"""MI355X-native UVA training step (drop-in for unified_video_action's hot path).

Product path: Python host layer on PyTorch-ROCm (device memory, streams,
torch.distributed) over libuva_hip.so (hand-written gfx950 HIP kernels, C ABI in
include/uva_hip.h).  There is no CPU fallback: every op fails loudly without the
library.
"""
__version__ = "0.1.0"
