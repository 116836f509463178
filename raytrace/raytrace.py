"""Alias of ray_trace_pb_amd.raytrace (drop-in import path ``raytrace.raytrace``)."""
from ray_trace_pb_amd.raytrace import *  # noqa: F401,F403
from ray_trace_pb_amd.raytrace import (Doublet, FlatSurface, PerfectLens, PlaneMirror, RefractingSurface,  # noqa: F401
                                       ReflectingSurface, SphericalSurface, Surface, System, dist_pt2plane,
                                       get_collimated_rays, get_free_space_abcd, get_ray_fan, intersect_rays,
                                       propagate_ray2plane, ray_angle_about_axis, trace_surfaces)
