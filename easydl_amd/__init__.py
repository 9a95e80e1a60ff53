"""easydl_amd — an MI355X-native elastic deep-learning training framework.

Capabilities of EasyDL (ElasticTrainer, ElasticOperator, Brain)
re-designed for single-node 8x MI355X (gfx950): PyTorch-ROCm + hand-written
HIP/CDNA4 kernels + RCCL over xGMI, with a native C++ runtime.
"""
__version__ = "0.1.0"
