"""Inter-stage transports (host / HIP IPC / RCCL) and multi-GPU helpers."""
