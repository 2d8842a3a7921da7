"""Multi-GPU sharding over torch.distributed (RCCL on ROCm, gloo on CPU)."""
