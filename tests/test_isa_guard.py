"""Guards on the generated gfx950 code of the engine's asm-issued gathers (CPU only).

k_rankB (visreps_amd/csrc/engine.hip) issues its TB-row gathers from inline asm and waits
for them with an asm `s_waitcnt`, which the compiler's waitcnt insertion cannot see
(ADVICE r2, medium). These tests read the built code object (tests/isa_check.py):

  * no instruction on any control-flow path touches a gather's destination VGPR between
    its issue and the `s_waitcnt vmcnt(N)` that retires it, and no path ends with one in
    flight;
  * the default forms (EST 0 exact, EST 2/3/4; B tie groups < 2^16) use no scratch: zero
    VGPR spills, zero private segment;
  * the checker itself flags a hand-made violating stream.
"""
import os
import re

import pytest

from isa_check import check_asm_gathers, check_object

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENGINE_O = os.path.join(ROOT, "visreps_amd", "csrc", "build", "engine.o")


@pytest.fixture(scope="module")
def rankb():
    if not os.path.exists(ENGINE_O):
        pytest.fail("visreps_amd/csrc/build/engine.o missing: run __graft_entry__.build() first")
    res = check_object(ENGINE_O, r"k_rankB")
    # (k_rankB_grid issues plain compiler-managed loads: no asm gathers to guard)
    res = {k: v for k, v in res.items() if "k_rankB_grid" not in k}
    assert len(res) >= 40, f"expected every k_rankB instantiation, found {len(res)}"
    return res


def _est(name: str) -> int:
    return int(re.search(r"k_rankBILb[01]ELb[01]E[tj]Lb[01]ELi(\d)E", name).group(1))


def test_asm_gathers_never_touched_in_flight(rankb):
    for name, r in rankb.items():
        assert r["asm_gathers"] >= 64, (name, r["asm_gathers"])
        assert not r["problems"], (name, r["problems"][:5])


def _bigt(name: str) -> bool:
    return re.search(r"k_rankBILb[01]ELb[01]E[tj]Lb([01])ELi\d", name).group(1) == "1"


def test_default_forms_have_no_scratch(rankb):
    for name, r in rankb.items():
        if _est(name) == 1:  # EST 1 (per-lane LDS table): selectable probe form, spills; dataflow-checked above
            continue
        if _bigt(name):  # B tie groups >= 2^16 (128-bit tie sums): a rare form, may spill a register or
            continue     # two around its segment loop; dataflow-checked above
        assert r["vgpr_spill_count"] == 0, (name, r)
        assert r["private_segment_fixed_size"] == 0, (name, r)


def test_checker_flags_sgpr_base_hazard():
    from isa_check import check_sgpr_base_hazards

    def code(lines):
        return [(4 * i, s, None) for i, s in enumerate(lines)]

    # round 5's fault: an SGPR spill restored by v_readlane right before an asm load's base
    bad = code(["v_readlane_b32 s1, v62, 7", "global_load_dwordx2 v[4:5], v0, s[0:1]"])
    assert check_sgpr_base_hazards(bad)
    # padded by 5 wait states, or written by the scalar unit: fine
    assert not check_sgpr_base_hazards(code(["v_readlane_b32 s1, v62, 7", "s_nop 4",
                                             "global_load_dwordx2 v[4:5], v0, s[0:1]"]))
    assert not check_sgpr_base_hazards(code(["v_readlane_b32 s40, v33, 17", "s_lshl_b64 s[16:17], s[40:41], 7",
                                             "s_add_u32 s16, s36, s16", "s_addc_u32 s17, s37, s17",
                                             "global_load_ushort v53, v31, s[16:17] nt"]))


def test_checker_flags_violations():
    def code(lines):
        return [(4 * i, s, None) for i, s in enumerate(lines)]

    ok = code(["global_load_ushort v10, v43, s[14:15] nt", "global_load_ushort v11, v43, s[16:17] nt",
               "v_add_u32_e32 v12, v13, v14", "s_waitcnt vmcnt(0)", "v_add_u32_e32 v12, v10, v11", "s_endpgm"])
    assert check_asm_gathers(ok) == (2, [])
    # a copy of an in-flight destination before its wait
    bad = code(["global_load_ushort v10, v43, s[14:15] nt", "v_mov_b32_e32 v20, v10", "s_waitcnt vmcnt(0)",
                "s_endpgm"])
    assert check_asm_gathers(bad)[1]
    # a spill store of it
    bad = code(["global_load_ushort v10, v43, s[14:15] nt", "scratch_store_dword off, v10, off",
                "s_waitcnt vmcnt(0)", "s_endpgm"])
    assert check_asm_gathers(bad)[1]
    # vmcnt(1) retires only the older of two loads: v11 is still in flight
    bad = code(["global_load_ushort v10, v43, s[14:15] nt", "global_load_ushort v11, v43, s[16:17] nt",
                "s_waitcnt vmcnt(1)", "v_add_u32_e32 v12, v10, v0", "v_add_u32_e32 v12, v11, v0",
                "s_waitcnt vmcnt(0)", "s_endpgm"])
    probs = check_asm_gathers(bad)[1]
    assert len(probs) == 1 and "v[11]" in probs[0]
    # a later compiler load makes the asm load older: vmcnt(1) then retires it
    ok = code(["global_load_ushort v10, v43, s[14:15] nt", "global_load_dword v30, v[2:3], off",
               "s_waitcnt vmcnt(1)", "v_add_u32_e32 v12, v10, v0", "s_endpgm"])
    assert check_asm_gathers(ok)[1] == []
    # a path that branches around the wait
    bad = [(0, "global_load_ushort v10, v43, s[14:15] nt", None), (4, "s_cbranch_scc1 2", 16),
           (8, "s_waitcnt vmcnt(0)", None), (12, "s_nop 0", None), (16, "v_add_u32_e32 v1, v10, v0", None),
           (20, "s_endpgm", None)]
    assert check_asm_gathers(bad)[1]


def test_grid_walks_have_no_hazards_or_scratch():
    # the region-fused walks (EST k_rankB_grid, exact k_rankB_gridx): no SGPR-base hazard on
    # their asm loads, and the exact grid walk -- 1-pair batches at 4 regions -- uses no scratch
    if not os.path.exists(ENGINE_O):
        pytest.fail("visreps_amd/csrc/build/engine.o missing: run __graft_entry__.build() first")
    res = check_object(ENGINE_O, r"k_rankB_grid")
    assert sum("k_rankB_gridx" in k for k in res) == 6, sorted(res)
    for name, r in res.items():
        assert not r["problems"], (name, r["problems"][:5])
        if "k_rankB_gridx" in name:
            assert r["vgpr_spill_count"] == 0 and r["private_segment_fixed_size"] == 0, (name, r)
