"""ISA audit of the HIP kernels (CPU: hipcc cross-compiles gfx950 here): no wide vector-memory store may have
its data registers overwritten by the very next instruction (tools/check_store_hazard.py — a hazard the
backend does not guard and which corrupted the on-chip RNN trainer's optimizer state on MI355X)."""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


@pytest.mark.skipif(not shutil.which("/opt/rocm/bin/hipcc"), reason="needs hipcc")
def test_no_wide_store_data_hazards():
    import check_store_hazard as chk

    assert chk.main(files=None) == 0


def test_checker_flags_the_pattern(tmp_path):
    import check_store_hazard as chk

    asm = tmp_path / "k.s"
    asm.write_text("\tbuffer_store_dwordx4 v[22:25], v42, s[36:39], s70 offen\n\tv_mov_b32_e32 v22, v32\n"
                   "\tglobal_store_dwordx4 v[0:1], v[4:7], off\n\ts_nop 0\n\tv_mov_b32_e32 v4, v1\n")
    hits = chk.scan(str(asm))
    assert len(hits) == 1 and "v22" in hits[0][1]


def test_checker_flags_asm_reading_a_fresh_mfma_result(tmp_path):
    import check_store_hazard as chk

    asm = tmp_path / "k.s"
    asm.write_text("\tv_mfma_f32_16x16x16_bf16 v[44:47], v[36:37], v[18:19], 0\n\tv_mov_b32_e32 v1, v2\n"
                   "\t;;#ASMSTART\n\tv_cndmask_b32 v44, 0, v44, s[24:25]\n\t;;#ASMEND\n"
                   "\tv_mfma_f32_16x16x16_bf16 v[8:11], v[36:37], v[18:19], 0\n\ts_nop 15\n\ts_nop 7\n"
                   "\t;;#ASMSTART\n\tv_cndmask_b32 v9, 0, v8, s[24:25]\n\t;;#ASMEND\n")
    hits = chk.scan_asm_mfma(str(asm))
    assert len(hits) == 1 and "v44" in hits[0][0] and hits[0][2] == 1
