"""Source guards for the HIP kernels (CPU, no GPU needed).

Inline asm that issues a memory instruction is invisible to the compiler's
hazard recognizer: round 4 tried a `global_store_dwordx4 ... sc1 nt` in asm
and the scheduler let VALUs rewrite the store's address and data VGPRs in the
next instructions with no wait states, which ended in an illegal-address
fault.  Kernel asm may only wait (`s_waitcnt`); every load,
store and atomic goes through a builtin the compiler schedules."""
import os
import re

import pytest

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "p4app-switchml_amd", "csrc")
ASM = re.compile(r"\basm\s*(?:volatile\s*)?\(\s*\"([^\"]*)\"", re.S)


def _kernel_sources():
    out = []
    for d, _, files in os.walk(CSRC):
        out += [os.path.join(d, f) for f in files if f.endswith((".hip", ".h"))]
    return sorted(out)


def test_kernel_sources_found():
    assert any(p.endswith("sml_quantizer.hip") for p in _kernel_sources())


@pytest.mark.parametrize("path", _kernel_sources(), ids=os.path.basename)
def test_inline_asm_only_waits(path):
    with open(path) as f:
        src = f.read()
    for m in ASM.finditer(src):
        body = m.group(1).strip()
        assert re.fullmatch(r"s_waitcnt(\s+(vmcnt|lgkmcnt|expcnt)\(\d+\))+", body), (
            f"{os.path.basename(path)}: inline asm {body!r} — memory instructions must go through "
            "compiler builtins (hazard wait states)")
