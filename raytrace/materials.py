"""Alias of ray_trace_pb_amd.materials (drop-in import path ``raytrace.materials``)."""
from ray_trace_pb_amd.materials import *  # noqa: F401,F403
from ray_trace_pb_amd.materials import Constant, Ebaf11, Material, Vacuum  # noqa: F401
