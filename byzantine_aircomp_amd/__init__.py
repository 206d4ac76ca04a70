"""MI355X-native geometric-median aggregation (Byzantine_AirComp hot path).

Drop-in replacements for the reference's aggregators, backed by hand-written
HIP kernels for gfx950 behind a C ABI (include/gmagg.h, libgmagg.so):

    from byzantine_aircomp_amd import gm2, gm, OMA

See DESIGN.md for the kernels and INTEGRATION.md for swapping them into the
reference's training loop.
"""
from .aggregators import (GMResult, Krum, OMA, context, gm, gm2, mean, median,  # noqa: F401
                          trimmed_mean)
from .panels import ClientPanels, panel_width  # noqa: F401

__version__ = "0.1.0"
