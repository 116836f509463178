"""Test infrastructure only: CPU restatements of the reference's ray-trace hot path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this
package -- as the checker / timed CPU baseline, never as part of the product path.
"""
