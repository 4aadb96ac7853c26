"""Library-GEMM selection for the Llama workload: PyTorch TunableOp over hipBLASLt / rocBLAS.

The projection GEMMs (≈70% of a Llama-3-8B training step, bench/gemm_bench.py) go to the ROCm
libraries.  hipBLASLt's default heuristic picks one kernel per shape; TunableOp instead times every
hipBLASLt and rocBLAS solution for each (op, transpose, M, N, K, dtype) the step actually issues and
keeps the fastest.  Tuning is done once on an MI355X (``mode="tune"``) and the winners are shipped in
``tuned/tunableop_mi355x.csv``; normal runs only read that table (``mode="use"``, the default when the
file exists).  The table carries TunableOp's own validators (PyTorch / ROCm / hipBLASLt versions, gfx
arch): on any other stack PyTorch refuses it and the default heuristic is used, so a stale table can
cost speed, never correctness.
"""
from __future__ import annotations

import os
from typing import Optional

import torch

__all__ = ["DEFAULT_TABLE", "setup_gemm_tuning"]

DEFAULT_TABLE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuned", "tunableop_mi355x.csv")


def setup_gemm_tuning(mode: str = "auto", path: Optional[str] = None, rank: int = 0) -> str:
    """Configure TunableOp before the first GEMM.  Returns the mode actually in effect.

    ``auto``: ``use`` if the table exists, else ``off``.  ``tune``: time all solutions for shapes not in
    the table and write the (merged) table; with several ranks each writes ``<path>.rank<r>``.
    """
    if not torch.cuda.is_available():
        return "off"
    path = path or DEFAULT_TABLE
    if mode == "auto":
        mode = "use" if os.path.exists(path) else "off"
    if mode == "off":
        return mode
    import torch.cuda.tunable as tunable

    tunable.enable(True)
    tunable.tuning_enable(mode == "tune")
    if mode == "tune":
        tunable.set_max_tuning_duration(10)  # ms per candidate solution (at least one timed call each)
        tunable.set_max_tuning_iterations(10)
        out = path if rank == 0 else f"{path}.rank{rank}"
        os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
        tunable.set_filename(out, False)
        if os.path.exists(path):
            tunable.read_file(path)
    else:
        tunable.set_filename(path, False)
        tunable.read_file(path)
    return mode
