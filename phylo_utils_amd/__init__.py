"""phylo_utils_amd -- MI355X (gfx950) Felsenstein pruning engine behind phylo_utils'
likelihood-engine seam.

The hot path (per-node partial updates over all site patterns, root combine,
lnL reduction) runs as hand-written HIP kernels in ``libphylo_hip.so`` reached
through a C ABI (``include/phylo_hip.h``).  Python here is the host mirror of the
reference interface: substitution and rate models, the post-order schedule,
alignment encoding, and ``TreeModel``.
"""
__version__ = "0.1.0"

from . import alignment, data, optimisation, rate_models, substitution_models, tree  # noqa: F401
from .discrete_gamma import discrete_gamma  # noqa: F401
from .tree_model import TreeModel  # noqa: F401
