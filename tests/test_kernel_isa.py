"""ISA regression guard for the hand-scheduled attention kernels (CPU: hipcc cross-compiles gfx950).

The properties the kernels' comments and profiles/r05_attn7 rely on, read from the assembly the build's
own flags produce (tools/isa.py): no scratch in the forward and dK/dV kernels, dK/dV's accumulators
pinned to AGPRs with no accumulator moves outside the epilogue, the forward at two waves per SIMD.  An
edit that makes the compiler spill or shuffle accumulators fails here, before any GPU run."""
import os
import shutil
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))

pytestmark = pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"),
                                reason="needs hipcc")


@pytest.fixture(scope="module")
def stats(tmp_path_factory):
    import isa

    out = str(tmp_path_factory.mktemp("isa") / "attention.s")
    st = isa.kernel_stats(os.path.join(REPO, "csrc", "ops", "attention.hip"), out=out)
    return {k: v for k, v in st.items()}


def _one(stats, needle):
    hits = [v for k, v in stats.items() if needle in k]
    assert len(hits) == 1, (needle, list(stats))
    return hits[0]


def test_one_production_kernel_per_attention_op(stats):
    names = sorted(k for k in stats if "gtk_attn" in k)
    assert len(names) == 4, names  # forward, backward pre-kernel, dK/dV, dQ


def test_forward_runs_two_waves_per_simd_without_scratch(stats):
    f = _one(stats, "attn_fwd2_kernel")
    assert f["Occupancy"] == 2 and f["ScratchSize"] == 0 and f["scratch"] == 0, f
    assert f["mfma"] == 64 and f["NumAgprs"] == 0, f


def test_dkdv_accumulators_stay_in_agprs(stats):
    k = _one(stats, "attn_bwd_dkdv_kernel")
    assert k["ScratchSize"] == 0 and k["scratch"] == 0, k
    assert k["NumAgprs"] == 128 and k["Occupancy"] == 1, k
    # 128 dV^T / dK^T accumulator registers read once in the epilogue, nothing moved inside the loop
    assert k["accvgpr_read"] + k["accvgpr_mov"] + k["accvgpr_write"] <= 256 + 1, k


def test_dq_spills_only_a_few_bytes(stats):
    q = _one(stats, "attn_bwd_dq2n_kernel")
    assert q["Occupancy"] == 2 and q["ScratchSize"] <= 64, q  # 48 B in the diagonal-tile code (profiles/r05_attn7)


@pytest.mark.parametrize("src", ["fused_ops.hip", "adamw_t.hip", "transpose.hip"])
def test_memory_bound_kernels_do_not_spill(tmp_path, src):
    """Every kernel of the Llama step's memory-bound sources is spill-free; the one exception is the
    RMSNorm backward instance for rows of 4097-8192 elements (NV = 16, not used by the Llama-3-8B /
    1B configs), whose next-row prefetch and per-lane dW columns exceed the register file."""
    import isa

    st = isa.kernel_stats(os.path.join(REPO, "csrc", "ops", src), out=str(tmp_path / "k.s"))
    assert st, src
    spilled = {k: v["ScratchSize"] for k, v in st.items() if v["ScratchSize"]}
    allowed = {k for k in spilled if "rmsnorm_bwd_kernelILi16E" in k}
    assert set(spilled) == allowed, spilled
