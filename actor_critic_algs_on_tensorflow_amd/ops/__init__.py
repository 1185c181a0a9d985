"""Op layer: each function dispatches GPU tensors to the hand-written HIP kernels (``torch.ops.acamd``) and CPU
tensors to the PyTorch reference implementation those kernels are tested against."""
from . import distributions, optim, returns
from .distributions import categorical_sample, gaussian_sample
from .optim import FlatParams, FusedAdam, FusedRMSprop
from .returns import PathAdv, gae, normalize_advantages, nstep_returns, path_adv

__all__ = ["distributions", "optim", "returns", "categorical_sample", "gaussian_sample", "FlatParams",
           "FusedAdam", "FusedRMSprop", "PathAdv", "gae", "normalize_advantages", "nstep_returns", "path_adv"]
