"""Static ISA checks of the detection kernel (CPU): the product build's assembly
(lcmap-firebird_amd/lib/ccd_kernels.s, written by `make isa-check`, which build() runs) has no
`if` join running under a narrowed EXEC with register-allocator work in it (the w4 divergence of
rounds 1-2), no inline-asm block clobbering a live SCC, and no unpadded wait-state
hazard around inline asm.  The checkers themselves are tested on hand-written snippets."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOLS = os.path.join(ROOT, 'tools')
ISA = os.path.join(ROOT, 'lcmap-firebird_amd', 'lib', 'ccd_kernels.s')
sys.path.insert(0, TOOLS)

import asm_scc_live  # noqa: E402
import dpp_hazards  # noqa: E402
import endcf_check  # noqa: E402

# the w4 reproducer's shape: an `if (l < NB)` lowered without an EXEC save whose join block
# received a spill reload (profiles/r03/w4_root_cause.md)
NARROWED_JOIN = '''_Zkernel:
	v_cmp_gt_i32_e32 vcc, 7, v16
	s_and_b64 s[16:17], exec, vcc
	v_mov_b32_dpp v2, v0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf bound_ctrl:1
	s_mov_b64 exec, s[16:17]
	s_cbranch_execz .LBB3_3307
; %bb.3306:
	v_sqrt_f64_e32 v[0:1], v[0:1]
	ds_write_b64 v2, v[0:1] offset:5760
.LBB3_3307:
	s_waitcnt lgkmcnt(0)
	scratch_load_dword v123, off, off offset:292 ; 4-byte Folded Reload
.LBB3_3308:
	s_or_b64 exec, exec, s[34:35]
	s_endpgm
'''

SAVED_JOIN = NARROWED_JOIN.replace('s_and_b64 s[16:17], exec, vcc', 's_and_saveexec_b64 s[18:19], vcc') \
    .replace('s_mov_b64 exec, s[16:17]\n', '') \
    .replace('.LBB3_3307:\n', '.LBB3_3307:\n\ts_or_b64 exec, exec, s[18:19]\n')

SCC_CLOBBER = '''_Zkernel:
	s_cmp_lt_u32 s4, s5
	;;#ASMSTART
	s_and_saveexec_b64 s[8:9], s[10:11]
	v_mul_f64 v[0:1], v[2:3], v[4:5]
	s_mov_b64 exec, s[8:9]
	;;#ASMEND
	s_cselect_b32 s6, 1, 0
	s_endpgm
'''


def _write(tmp_path, text):
    p = tmp_path / 'k.s'
    p.write_text(text)
    return str(p)


def test_endcf_check_finds_the_narrowed_join(tmp_path, capsys):
    assert endcf_check.main(_write(tmp_path, NARROWED_JOIN)) == 1
    assert 'scratch_load_dword v123' in capsys.readouterr().out
    assert endcf_check.main(_write(tmp_path, SAVED_JOIN)) == 0


def test_scc_checker_finds_a_clobbered_scc(tmp_path):
    assert asm_scc_live.main(_write(tmp_path, SCC_CLOBBER)) == 1
    assert asm_scc_live.main(_write(tmp_path, SCC_CLOBBER.replace('s_cselect_b32 s6, 1, 0', 's_cmp_eq_u32 s4, 0\n\ts_cselect_b32 s6, 1, 0'))) == 0


def test_hazard_checker_rules(tmp_path):
    snippet = '''_Zkernel:
	v_add_f64 v[0:1], v[2:3], v[4:5]
	v_mov_b32_dpp v6, v0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf
	v_rcp_f64_e32 v[8:9], v[10:11]
	v_mul_f64 v[12:13], v[8:9], v[8:9]
	v_readfirstlane_b32 s4, v12
	v_readlane_b32 s5, v14, s4
	v_cmpx_gt_f32_e32 vcc, v1, v2
	v_mov_b32_dpp v7, v3 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf
	v_readfirstlane_b32 s8, v20
	global_load_dword v30, v31, s[8:9]
	v_div_scale_f64 v[40:41], vcc, v[42:43], v[42:43], v[44:45]
	v_div_fmas_f64 v[40:41], v[40:41], v[46:47], v[48:49]
'''
    assert dpp_hazards.main(_write(tmp_path, snippet), all_hazards=True) == 7
    padded = snippet.replace('\tv_mov_b32_dpp v6', '\ts_nop 1\n\tv_mov_b32_dpp v6')
    assert dpp_hazards.main(_write(tmp_path, padded), all_hazards=True) == 6
    # inline-asm scope: compiler-only hazards are not reported by default
    assert dpp_hazards.main(_write(tmp_path, snippet)) == 0


@pytest.mark.skipif(not os.path.exists(ISA), reason='lib/ccd_kernels.s not built (make -C lcmap-firebird_amd isa-check)')
def test_product_isa_is_clean():
    for tool in ('endcf_check.py', 'asm_scc_live.py'):
        r = subprocess.run([sys.executable, os.path.join(TOOLS, tool), ISA, 'ccd_detect'], capture_output=True, text=True)
        assert r.returncode == 0, r.stdout[-2000:]
    r = subprocess.run([sys.executable, os.path.join(TOOLS, 'dpp_hazards.py'), ISA], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-2000:]
    # the build carries the fix: no `if` is lowered without saving EXEC
    for kern in ('ccd_detect_w4', 'ccd_detect_w3'):  # the product's 4-waves kernel, and w3
        out = subprocess.run([sys.executable, os.path.join(TOOLS, 'endcf_check.py'), ISA, kern],
                             capture_output=True, text=True).stdout
        assert ': 0 ifs without an EXEC save' in out, out
