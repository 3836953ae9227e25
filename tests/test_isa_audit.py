"""ISA audits of the production render kernels (CPU: hipcc cross-compiles gfx950 assembly).

1. Wide buffer stores.  A buffer store of more than 64 bits whose data VGPRs are overwritten by
   the very next VALU instruction loses the overwritten dwords on gfx950, and the compiler adds
   no wait state when the store's soffset is an SGPR.  That was round 2's "stale path-state read"
   (b128 path-state stores; DESIGN.md §4 "path state"): the kernel now stores path state with 8-B
   stores, and this test keeps any wide SGPR-soffset store followed by such a write out of the
   shipped code (tools/isa_audit.py).
2. Load waits.  Every vector-memory load's destination is covered by an s_waitcnt vmcnt before
   its first use on every fall-through / branch path (tools/waitcnt_audit.py).
"""
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tools"))
import isa_audit  # noqa: E402
import waitcnt_audit  # noqa: E402

# the production kernels (no scratch): the static walk of the diagnostic variants, which spill 50-250
# VGPRs to scratch, reaches spill reloads through infeasible exec-mask paths (reports that the
# branch-insensitive walk cannot rule out), so the load-wait audit covers the shipped variants
# (one-sample and sample-group instances of both stack rings)
WAIT_VARIANTS = ["ILi4ELb0ELb0ELi8ELb0EE", "ILi4ELb0ELb0ELi16ELb0EE", "ILi4ELb0ELb0ELi8ELb1EE", "ILi4ELb0ELb0ELi16ELb1EE"]


@pytest.fixture(scope="module")
def kernel_asm(tmp_path_factory):
    out = tmp_path_factory.mktemp("isa") / "rt_render.s"
    subprocess.run(["make", "-s", "-C", str(ROOT / "my-raytracer_amd"), "asm", f"ASM_OUT={out}"], check=True,
                   capture_output=True, timeout=900)
    return out


def test_no_wide_store_overwrite_hazard(kernel_asm):
    sites = isa_audit.audit(kernel_asm.read_text())
    assert sites == [], sites[:5]


@pytest.mark.parametrize("variant", WAIT_VARIANTS)
def test_every_load_waited_for_before_use(kernel_asm, variant):
    body = waitcnt_audit.kernel_lines(str(kernel_asm), variant)
    checked, problems = waitcnt_audit.audit(body)
    assert checked > 50
    assert problems == [], problems[:5]


def test_audit_finds_the_round2_hazard_pattern():
    # the exact sequence of the failing build: a b128 path-state store with an SGPR soffset, then a
    # VALU write of one of its data VGPRs
    text = "\n".join(["_Zkernel:", "\tbuffer_store_dwordx4 v[6:9], v102, s[12:15], s10 offen",
                      "\tv_sub_u32_e32 v7, 0, v68", "\tbuffer_store_dwordx4 v[6:9], v102, s[12:15], 16 offen",
                      "\tv_sub_u32_e32 v7, 0, v68", "\tbuffer_store_dwordx4 v[6:9], v102, s[12:15], s10 offen",
                      "\ts_nop 0", "\tv_sub_u32_e32 v7, 0, v68", "\tbuffer_store_dwordx2 v[6:7], v102, s[12:15], s10 offen",
                      "\tv_sub_u32_e32 v7, 0, v68"])
    sites = isa_audit.audit(text)
    assert len(sites) == 1 and "s10" in sites[0][2]


def test_waitcnt_audit_flags_missing_wait_and_skips_flag_decided_paths():
    # a use of a loaded register with no s_waitcnt vmcnt on the path is reported ...
    bad = ["\tglobal_load_dwordx2 v[14:15], v[2:3], off", "\tv_mov_b32_e32 v1, v14", "\ts_endpgm"]
    assert waitcnt_audit.audit(bad)[1]
    # ... a use reached only through a branch pair whose flag rules it out is not (both image-store
    # blocks skipped: s[6:7] = -1 makes "s_andn2_b64 vcc, exec, s[6:7]; s_cbranch_vccnz" fall through)
    ok = ["\tglobal_load_dwordx2 v[14:15], v[2:3], off", "\ts_mov_b64 s[6:7], -1",
          "\ts_and_b64 vcc, exec, s[18:19]", "\ts_cbranch_vccz .LBB0_2",
          "\ts_waitcnt vmcnt(0)", "\tflat_store_dwordx2 v[4:5], v[14:15]", "\ts_mov_b64 s[6:7], 0",
          ".LBB0_2:", "\ts_andn2_b64 vcc, exec, s[6:7]", "\ts_cbranch_vccnz .LBB0_3",
          "\ts_waitcnt vmcnt(0)", "\tflat_store_dwordx2 v[4:5], v[14:15]",
          ".LBB0_3:", "\tv_mov_b32_e32 v1, v14", "\ts_endpgm"]
    assert waitcnt_audit.audit(ok)[1] == []
