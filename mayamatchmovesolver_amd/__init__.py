"""MI355X-native bundle-adjustment core for mmSolver's LM hot path.

The shipped compute path is ``csrc/libmmba.so`` (hand-written HIP for gfx950
behind the C ABI in ``include/mmba.h``); this package is the host-side mirror
of the reference's solver interface: problem assembly (``problem``), options
(``options``), the ABI binding (``_lib``) and the solve entry point
(``solver``).
"""
from . import abi  # noqa: F401
from .options import make_options  # noqa: F401
from .problem import Problem, SceneBuilder, AttrRef  # noqa: F401

__all__ = ["abi", "make_options", "Problem", "SceneBuilder", "AttrRef"]
