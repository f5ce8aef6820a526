"""Profiling: roctracer kernel-activity bridge (``tracer``)."""
