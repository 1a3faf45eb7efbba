"""gsr_train -- the training step around the rasterizer, MI355X-native.

GaussianModel mirrors scene/gaussian_model.py on one device arena; GaussianAdam is
the fused replacement of its torch.optim.Adam.  Kernels: include/gsr_train.h
(libgsr.so, csrc/train.hip)."""
from .gaussian_model import GaussianModel, get_expon_lr_func, inverse_sigmoid, build_rotation  # noqa: F401
from .optim import GaussianAdam  # noqa: F401
from ._C import ArenaSpec  # noqa: F401
from .knn import distCUDA2  # noqa: F401
