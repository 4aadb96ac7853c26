"""Model families: the Llama-3 validation workload (BASELINE config 5)."""
from .llama import FlatParams, Llama, LlamaConfig, smoke_step
from .optim import FlatAdamW
from .checkpoint import CheckpointWriter, load_checkpoint

__all__ = ["FlatParams", "Llama", "LlamaConfig", "smoke_step", "FlatAdamW", "CheckpointWriter", "load_checkpoint"]
