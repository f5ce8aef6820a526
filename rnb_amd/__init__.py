"""rnb_amd -- Replicate-and-Batch video inference engine for AMD MI355X.

A new implementation of the capabilities of snuspl/rnb designed for CDNA4:
pipelines of replicated runner processes (one HIP stream each) joined by
queues and producer-owned HBM slot rings (HIP IPC / RCCL), an R(2+1)D engine
built on hand-written MFMA kernels (``rnb_amd.ops``), and a roctracer kernel
tracer (``rnb_amd.profiling``).
"""
__version__ = "0.1.0"
