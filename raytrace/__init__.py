"""Import alias so code written against the reference (``import raytrace.raytrace as rt``,
``from raytrace.materials import Bk7``) runs unchanged on ray_trace_pb_amd."""
from ray_trace_pb_amd import __version__  # noqa: F401
