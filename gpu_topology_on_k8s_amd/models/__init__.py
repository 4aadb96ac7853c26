"""Model families: the Llama-3 validation workload (BASELINE config 5)."""
from .llama import FlatParams, Llama, LlamaConfig, smoke_step
from .optim import FlatAdamW

__all__ = ["FlatParams", "Llama", "LlamaConfig", "smoke_step", "FlatAdamW"]
