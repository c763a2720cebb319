"""euler_amd — an MI355X-native large-scale graph-learning framework with the
capabilities of Euler-2.0 (renyi533/euler): C++ sharded graph engine + GQL,
tf_euler-shaped Python API on PyTorch-ROCm, gfx950 HIP message-passing kernels and
RCCL data/embedding parallelism."""
__version__ = "0.1.0"
