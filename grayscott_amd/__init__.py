"""grayscott_amd -- an MI355X-native 3D Gray-Scott reaction-diffusion framework.

Same capabilities and config surface as GrayScott.jl (reference snapshot 2025-01-03), built
MI355X-first: hand-written gfx950 HIP stencil kernels, RCCL halo exchange over xGMI, a native
C++ scheduler, a native BP4 writer, and a torch.distributed control plane.
"""
__version__ = "0.1.0"

from .utils.config import Settings, get_settings, load_settings, parse_settings_toml  # noqa: F401
from .parallel.decomp import CartDomain, dims_create, init_domain  # noqa: F401
