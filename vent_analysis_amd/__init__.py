"""vent_analysis_amd -- MI355X-native (gfx950 HIP) implementation of the Vent_Analysis voxel hot
path: N4 bias correction, mean-anchored / linear-binning / k-means VDP, defect morphology and the
cluster index, behind the reference's ``Vent_Analysis`` class and ``CI`` module surface.

    from vent_analysis_amd import Vent_Analysis      # drop-in for Vent_Analysis.Vent_Analysis
    from vent_analysis_amd import CI                 # drop-in for the reference CI module
"""
from .Vent_Analysis import Vent_Analysis  # noqa: F401
from . import CI  # noqa: F401

__version__ = "0.1.0"
