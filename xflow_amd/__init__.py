"""xflow-amd: an MI355X-native sparse CTR training engine with the
capabilities of liuhatry/xflow (LR / FM / MVM with FTRL-Proximal or SGD over
hashed libffm features), built on PyTorch-ROCm, hand-written gfx950 HIP
kernels and RCCL over xGMI.

The ps-lite parameter server of the reference becomes an open-addressing hash
table resident in GPU HBM and sharded across the node's GPUs; Pull/Push are
sparse all-to-alls.  See docs/DESIGN.md.
"""
__version__ = "0.1.0"

from xflow_amd.config import (EngineConfig, ModelConfig, OptimConfig,  # noqa: F401
                              TrainConfig)
