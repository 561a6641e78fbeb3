"""Static checks on the gfx950 code objects of the built library (no GPU needed).

The bootstrap engine's B walk (visreps_amd/csrc/engine.hip, k_rankB) issues its TB-row
gathers through inline asm (`global_load_* vD, vOff, s[base]`, the saddr form) and waits
for them with an asm `s_waitcnt`. The compiler's waitcnt insertion cannot see loads
issued from asm, so correctness needs two things of the generated code:

  1. no compiler-generated instruction reads, writes, copies or spills a destination
     VGPR of an asm gather between its issue and the `s_waitcnt vmcnt(N)` that retires
     it (vmcnt retires the oldest vector-memory ops first; loads, stores and scratch ops
     count together), and no branch leaves that straight-line stretch;
  2. no scratch at all in those kernels (`.vgpr_spill_count == 0`,
     `.private_segment_fixed_size == 0`): a spill is a compiler-inserted VMEM op that
     could land anywhere in the stretch.

`check_object(path)` extracts the gfx950 code object from a hipcc `.o`, disassembles it
with the ROCm llvm tools and returns the per-kernel findings.
"""
from __future__ import annotations

import os
import re
import subprocess
import tempfile

import yaml

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"

_VMEM = re.compile(r"^(global_|buffer_|scratch_|flat_)")
# asm gather form: saddr global load, `global_load_<t> vD, vOff, s[a:b]`
_SADDR_LOAD = re.compile(r"^global_load_\w+\s+(v\d+|v\[\d+:\d+\]),\s*v\d+,\s*s\[\d+:\d+\]")
_VREG = re.compile(r"\bv(\d+)\b|\bv\[(\d+):(\d+)\]")
_FUNC = re.compile(r"^[0-9a-f]+ <(\S+)>:$")


def _regs(text: str) -> set[int]:
    out: set[int] = set()
    for m in _VREG.finditer(text):
        if m.group(1) is not None:
            out.add(int(m.group(1)))
        else:
            out.update(range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def extract_code_object(obj: str, out_dir: str) -> str:
    fat = os.path.join(out_dir, "fatbin.bin")
    co = os.path.join(out_dir, "gfx950.co")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj, os.path.join(out_dir, "x.o")],
                   check=True, capture_output=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--targets={TARGET}",
                    f"--input={fat}", f"--output={co}"], check=True, capture_output=True)
    return co


def kernel_metadata(co: str) -> dict[str, dict]:
    txt = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                         text=True).stdout
    body = txt[txt.index("amdhsa.kernels:"):]
    body = body[:body.index("\n...")] if "\n..." in body else body
    meta = yaml.safe_load(body)
    return {k[".name"]: k for k in meta["amdhsa.kernels"]}


def disassemble(co: str) -> dict[str, list[tuple[int, str, int | None]]]:
    """Per kernel: (address, instruction text, branch target address or None)."""
    txt = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], check=True,
                         capture_output=True, text=True).stdout
    funcs: dict[str, list] = {}
    base: dict[str, int] = {}
    cur = None
    for line in txt.splitlines():
        m = _FUNC.match(line.strip())
        if m:
            cur = funcs.setdefault(m.group(1), [])
            base[m.group(1)] = int(line.split()[0], 16)
            continue
        if cur is None or "//" not in line:
            continue
        ins, comment = line.split("//", 1)
        ins = ins.strip()
        if not ins:
            continue
        addr = int(comment.strip().split(":")[0], 16)
        tgt = None
        t = re.search(r"<(\S+)\+0x([0-9a-f]+)>", comment)
        if t and t.group(1) in base:
            tgt = base[t.group(1)] + int(t.group(2), 16)
        cur.append((addr, ins, tgt))
    return funcs


def check_asm_gathers(code: list[tuple[int, str, int | None]]) -> tuple[int, list[str]]:
    """Forward dataflow over the kernel's control-flow graph. The state at an instruction is
    the set of asm gathers still in flight, each with the count of vector-memory ops issued
    after it (`s_waitcnt vmcnt(N)` retires exactly those with N or more younger ops; older
    compiler loads never change that, so they need no tracking). Returns (number of asm
    gathers in the kernel, problems)."""
    index = {a: i for i, (a, _, _) in enumerate(code)}
    n_gathers = sum(1 for _, ins, _ in code if _SADDR_LOAD.match(ins))
    problems: list[str] = []
    seen: set[tuple[int, tuple]] = set()
    work = [(0, ())]
    while work:
        i, state = work.pop()
        while i < len(code):
            if (i, state) in seen:
                break
            seen.add((i, state))
            addr, ins, tgt = code[i]
            op = ins.split()[0]
            if state:
                pending = set().union(*[e[0] for e in state])
                used = _regs(ins.split(None, 1)[1]) if " " in ins else set()
                hit = used & pending
                if hit and op != "s_waitcnt":
                    problems.append(f"{addr:#x} `{ins}`: touches in-flight asm gather register(s) v{sorted(hit)}")
            if op == "s_waitcnt":
                m = re.search(r"vmcnt\((\d+)\)", ins)
                if m:
                    keep = int(m.group(1))
                    state = tuple(e for e in state if e[1] < keep)
            elif _VMEM.match(op):
                # at most 63 vector-memory ops are outstanding (6-bit vmcnt): one with 63
                # younger ones has completed -- this also bounds the states around loops
                state = tuple((e[0], e[1] + 1, e[2]) for e in state if e[1] + 1 < 63)
                gm = _SADDR_LOAD.match(ins)
                if gm:
                    # the flag: a streaming (nt) load, i.e. a TB row gather
                    state = state + ((frozenset(_regs(gm.group(1))), 0, ins.rstrip().endswith(" nt")),)
            if op == "s_endpgm":
                # a TB row gather still in flight at the end (other saddr loads may be compiler
                # loads whose value a path never uses: legal, the wave's end waits for them)
                if any(e[2] for e in state):
                    problems.append(f"{addr:#x}: kernel ends with asm gathers in flight")
                break
            if op.startswith(("s_setpc", "s_swappc")):
                if state:
                    problems.append(f"{addr:#x} `{ins}`: indirect jump with asm gathers in flight")
                break
            if op.startswith("s_cbranch") or op == "s_branch":
                if tgt is None or tgt not in index:
                    if state:
                        problems.append(f"{addr:#x} `{ins}`: unresolved branch with asm gathers in flight")
                else:
                    work.append((index[tgt], state))
                if op == "s_branch":
                    break
            i += 1
    return n_gathers, sorted(set(problems))


_SREG = re.compile(r"\bs(\d+)\b|\bs\[(\d+):(\d+)\]")
_SADDR_ANY = re.compile(r"^global_(load|store)\w*\s+.*,\s*(s\[\d+:\d+\])(\s|$)")


def _sregs(text: str) -> set[int]:
    out: set[int] = set()
    for m in _SREG.finditer(text):
        if m.group(1) is not None:
            out.add(int(m.group(1)))
        else:
            out.update(range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def check_sgpr_base_hazards(code: list[tuple[int, str, int | None]], wait_states: int = 5) -> list[str]:
    """A VALU write of an SGPR (v_readlane / v_readfirstlane, or an SGPR spill restored from
    a VGPR lane) followed within `wait_states` wait states by a vector-memory instruction
    reading that SGPR as its scalar base: the hardware needs 5 wait states there, hipcc pads
    its own loads but not the inside of an asm statement (cdna_hip_programming.md §5.7
    item 2), and the load then forms its address from the SGPR's stale value. Round 5's
    MEMORY_APERTURE_VIOLATION in k_rankB (masks from L2, the VR_XW_SLO probe build: 32 SGPRs
    spilled to VGPR lanes) was this: `v_readlane_b32 s1, v62, 7` restoring the mask table's
    address high word right before the asm `global_load_dwordx2 v[4:5], v0, s[0:1]`.
    Straight-line look-back (a branch target in the window is treated as a fresh start)."""
    problems = []
    targets = {t for _, _, t in code if t is not None}
    for i, (addr, ins, _) in enumerate(code):
        m = _SADDR_ANY.match(ins)
        if not m:
            continue
        base = _sregs(m.group(2))
        ws = 0
        for k in range(i - 1, -1, -1):
            a_k, t_k, _ = code[k]
            op = t_k.split()[0]
            if op == "s_nop":
                ws += int(t_k.split()[1], 0) + 1
            else:
                dst = t_k.split(None, 1)[1].split(",")[0] if " " in t_k else ""
                if _sregs(dst) & base:
                    if op.startswith("v_") and ws < wait_states:
                        problems.append(f"{addr:#x} `{ins}`: base written by `{t_k}` {ws} wait states before")
                    break
                ws += 1
            if ws >= wait_states or a_k in targets:
                break
    return problems


def check_object(obj: str, kernel_pattern: str) -> dict[str, dict]:
    """Findings for every kernel whose symbol matches kernel_pattern."""
    with tempfile.TemporaryDirectory() as d:
        co = extract_code_object(obj, d)
        meta = kernel_metadata(co)
        code = disassemble(co)
    out = {}
    pat = re.compile(kernel_pattern)
    for name, md in meta.items():
        if not pat.search(name):
            continue
        n, probs = check_asm_gathers(code.get(name, []))
        probs = probs + check_sgpr_base_hazards(code.get(name, []))
        out[name] = {"vgpr_spill_count": md.get(".vgpr_spill_count", 0),
                     "sgpr_spill_count": md.get(".sgpr_spill_count", 0),
                     "private_segment_fixed_size": md.get(".private_segment_fixed_size", 0),
                     "vgpr_count": md.get(".vgpr_count"), "asm_gathers": n, "problems": probs,
                     "instructions": len(code.get(name, []))}
    return out


if __name__ == "__main__":
    import sys

    res = check_object(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "k_rankB")
    for k, v in res.items():
        print(k[:70], {x: y for x, y in v.items() if x != "problems"}, len(v["problems"]))
        for p in v["problems"][:5]:
            print("   ", p)
