"""The inline-asm MFMA kernels (attn_fwd3 / attn_dq2 / attn_dkdv2) read no
accumulator before its MFMA has landed and spill nothing (tools/asm_hazards.py: the
compiler does not see an asm MFMA's latency, so a copy or spill it places right after one
reads the old value -- the failure the first attn_fwd3 build had).  CPU only: hipcc -S."""
import os
import shutil
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


@pytest.mark.skipif(shutil.which("/opt/rocm/bin/hipcc") is None, reason="no hipcc")
def test_asm_mfma_kernels_have_no_accumulator_hazards():
    import asm_hazards
    res = asm_hazards.scan(asm_hazards.build_asm("attn_bf16_dq2"))
    assert res, "no asm-MFMA kernels found"
    bad = {k: v for k, v in res.items() if v["hazards"] or v["scratch"]}
    assert not bad, bad
