"""Static checks of the compiled gfx950 kernels (CPU container: hipcc cross-compiles).

The protein kernel's P prefetches are inline-asm loads waited for with counted
`s_waitcnt vmcnt(N)` (pu_kernels.hip, k_prune_mfma).  The compiler cannot see that those
registers fill asynchronously, so this walks the generated ISA and fails if any instruction
touches a prefetch register before its wait (scripts/check_async_regs.py), and checks the
register budget that sets the kernel's occupancy.
"""
import os
import re
import shutil
import subprocess
import sys

import pytest

from conftest import ROOT

HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
SRC = os.path.join(ROOT, "phylo_utils_amd", "csrc", "pu_kernels.hip")

pytestmark = pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")


@pytest.fixture(scope="module")
def isa(tmp_path_factory):
    out = tmp_path_factory.mktemp("isa") / "pu_kernels.s"
    # same device flags as phylo_utils_amd/csrc/Makefile
    cmd = [HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "-mllvm",
           "-simplifycfg-sink-common=false", "-S", "--cuda-device-only", SRC, "-o", str(out)]
    subprocess.run(cmd, check=True, capture_output=True, timeout=600)
    return str(out)


def test_no_prefetch_register_touched_before_its_wait(isa):
    script = os.path.join(ROOT, "scripts", "check_async_regs.py")
    r = subprocess.run([sys.executable, script, isa, "k_prune_mfma"], capture_output=True,
                       text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    # {coded, dense} x {LNL, KEEP, generic, LNL chain task, KEEP chain task}
    assert r.stdout.count("0 hazard(s)") == 10


def test_protein_kernel_register_budget(isa):
    text = open(isa).read()
    metas = re.findall(r"\.agpr_count:\s+(\d+)\s*\n(?:.*\n){0,64}?\s+\.name:\s+(\S*k_prune_mfma\S*)"
                       r"(?:.*\n){0,40}?\s+\.vgpr_count:\s+(\d+)", text)
    assert len(metas) == 10
    for agpr, name, vgpr in metas:
        # 3 waves per SIMD: at most 168 unified registers, no scratch spills
        assert int(vgpr) + int(agpr) <= 168, (name, vgpr, agpr)
    assert ".vgpr_spill_count: 0" in text


def test_traversal_kernels_use_no_scratch(isa):
    """Every shipped traversal kernel (k_prune, k_prune_mfma) keeps its state in registers and
    LDS: no private segment and no scratch or flat instruction.  r04's register stash slots
    (TV_RSLOTS) were an array reached through a pointer and lived in scratch (88 bytes per
    lane, scratch stores in the op loop, flat loads where a select mixed them with the LDS
    stash); r05 keeps them as named registers (RegStash), and the spilling 7- / 8-wave builds
    are gone."""
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    from kernel_resources import kernels
    ks = {n: r for n, r in kernels(open(isa).read()).items() if "k_prune" in n}
    assert len(ks) >= 40, sorted(ks)
    bad = {n: r for n, r in ks.items()
           if r["private"] != 0 or r["scratch_insts"] or r["flat_insts"]}
    assert not bad, bad
