"""ray_trace_pb_amd -- MI355X-native sequential optical ray tracer.

Drop-in for the ``raytrace`` package of QI2lab/ray_trace_pb: ``ray_trace_pb_amd.raytrace`` and
``ray_trace_pb_amd.materials`` expose the same API (also importable as ``raytrace.raytrace`` /
``raytrace.materials`` through the alias package at the repository root).  ``System.ray_trace`` runs
on gfx950 through the C ABI of include/rtpb.h (librtpb.so, built in-tree).
"""
__version__ = "0.1.0"

from . import materials, raytrace  # noqa: F401
