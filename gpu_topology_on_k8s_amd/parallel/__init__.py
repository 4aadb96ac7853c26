"""Collectives and data parallelism over RCCL/xGMI."""
