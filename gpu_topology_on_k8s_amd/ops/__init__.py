"""Native ops: HIP link probe (K1-K4) and fused Llama kernels."""
