"""Device-assembly hazard check (CPU: hipcc -S for gfx950, no GPU).

A scalar load whose destination registers overlap the address registers of a later scalar load
issued before the lgkmcnt wait is a race: if the first load returns early, the second one reads
loaded data as its address. Inline asm with non-early-clobber outputs produced exactly that
(trace.h load_inner_uniform, rounds 4-5: rare MEMORY_APERTURE_VIOLATION faults).
This test compiles the shipping kernels to assembly and scans every s_load sequence."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"
SLOAD = re.compile(r"^\s*s_load_dword\w*\s+s\[(\d+):(\d+)\],\s+s\[(\d+):(\d+)\]")
SLOAD1 = re.compile(r"^\s*s_load_dword\s+s(\d+),\s+s\[(\d+):(\d+)\]")


def hazards(asm_text):
    """(line, text) of every scalar load reading an address register that an earlier scalar load of
    the same unwaited group writes."""
    out = []
    pending = set()  # SGPRs written by scalar loads not yet waited for
    for i, line in enumerate(asm_text.splitlines(), 1):
        s = line.strip()
        if s.startswith("s_waitcnt") and "lgkmcnt(0)" in s:
            pending.clear()
            continue
        if re.match(r"^[\w.$]+:", s) or s.startswith("s_cbranch") or s.startswith("s_branch") or s.startswith("s_setpc"):
            pending.clear()  # control flow: the group ends (the compiler waits before uses)
            continue
        m = SLOAD.match(line)
        if m:
            d0, d1, a0, a1 = map(int, m.groups())
            if pending & {a0, a1}:
                out.append((i, s))
            pending |= set(range(d0, d1 + 1))
            continue
        m = SLOAD1.match(line)
        if m:
            d, a0, a1 = map(int, m.groups())
            if pending & {a0, a1}:
                out.append((i, s))
            pending.add(d)
    return out


def test_hazard_scanner():
    bad = "s_load_dwordx8 s[12:19], s[12:13], 0x0\n s_load_dwordx4 s[24:27], s[12:13], 0x20\n"
    good = "s_load_dwordx8 s[16:23], s[12:13], 0x0\n s_load_dwordx4 s[24:27], s[12:13], 0x20\n"
    waited = "s_load_dwordx2 s[12:13], s[4:5], 0x0\n s_waitcnt lgkmcnt(0)\n s_load_dwordx4 s[24:27], s[12:13], 0x0\n"
    assert hazards(bad) and not hazards(good) and not hazards(waited)


@pytest.mark.parametrize("src", ["render.hip", "paths.hip"])
def test_shipping_kernels_have_no_scalar_load_address_race(src, tmp_path):
    if not os.path.exists(HIPCC):
        pytest.skip("no ROCm compiler")
    out = tmp_path / (src + ".s")
    cmd = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math",
           "--cuda-device-only", "-S", "-o", str(out), os.path.join(ROOT, "atray_amd", "csrc", src)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    bad = hazards(out.read_text())
    assert not bad, "\n".join(f"{src}.s:{i}: {s}" for i, s in bad[:10])
