"""lfit_python_amd -- MI355X-native CV eclipse light-curve evaluator.

A drop-in for the lfit.CV.calcFlux() hot path of wildjames/lfit_python:
hand-written gfx950 HIP kernels (FP64) behind a C ABI (include/lfg.h),
driven from Python with PyTorch-ROCm tensors.

    lfit.CV / lfit.flux_batch    lfit.CV replacement (scalar / batched)
    roche                        trm.roche primitives on the GPU
    tree, cvmodel                the reference's model tree and input format
    batch                        compiled tree -> batched ln_prob on device
    sampler                      device-resident emcee stretch-move ensemble
"""
from . import _native  # noqa: F401

__version__ = "0.1.0"


def build(force=False):
    """Compile the HIP library in-tree for gfx950."""
    return _native.build(force=force)
