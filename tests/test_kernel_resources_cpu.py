"""CPU check of the built gfx950 code objects: no kernel of the library spills
VGPRs or uses scratch memory.  A VGPR spill is silent (results stay exact) but
costs HBM traffic the PMC passes then count -- it happened once (a lane-held
length check pushed the PerBlock/Prefix decode modes past their VGPR budget:
12 B/lane of scratch, C3 WRITE_SIZE +3%).  Reads the AMDGPU
metadata of the gfx950 code object inside each compiled HIP object
(turbopfor-cpp_amd/build/*.o, .hip_fatbin section); no GPU needed.
SGPR spills are allowed: they go to VGPR lanes (v_writelane), not memory --
the generic decoder caps its SGPRs at 80 on purpose.  The
rejected pipelined encoder (k_enc256v32_pipe, measurement-only probe modes
>= 16) is exempt."""
import glob
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "turbopfor-cpp_amd", "build")
LLVM = "/opt/rocm/lib/llvm/bin"
HIP_OBJS = [os.path.join(BUILD, os.path.basename(f)[:-4] + ".o")
            for f in glob.glob(os.path.join(ROOT, "turbopfor-cpp_amd", "csrc", "*.hip"))]


def kernels_of(obj, tmp):
    bundle, co = os.path.join(tmp, "x.bundle"), os.path.join(tmp, "x.co")
    subprocess.check_call(["objcopy", "--dump-section", f".hip_fatbin={bundle}", obj])
    subprocess.check_call([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                           "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={bundle}", f"--output={co}"])
    notes = subprocess.check_output([os.path.join(LLVM, "llvm-readelf"), "--notes", co]).decode()
    out, name = {}, None
    for line in notes.splitlines():
        m = re.search(r"\.name:\s+(_Z\S+)", line)
        if m:
            name = m.group(1)
        m = re.search(r"\.(private_segment_fixed_size|vgpr_spill_count|sgpr_spill_count):\s+(\d+)", line)
        if m and name:
            out.setdefault(name, {})[m.group(1)] = int(m.group(2))
    return out


@pytest.mark.skipif(not os.path.isdir(LLVM) or shutil.which("objcopy") is None, reason="ROCm llvm tools / objcopy absent")
@pytest.mark.parametrize("obj", HIP_OBJS, ids=[os.path.basename(o) for o in HIP_OBJS])
def test_no_kernel_spills(obj, tmp_path):
    if not os.path.exists(obj):
        pytest.skip("library not built (python -c 'import __graft_entry__ as g; g.build()')")
    ks = kernels_of(obj, str(tmp_path))
    assert ks, f"no kernel metadata found in {obj}"
    bad = {k: v for k, v in ks.items() if "k_enc256v32_pipe" not in k
           and any(v.get(f, 0) for f in ("private_segment_fixed_size", "vgpr_spill_count"))}
    assert not bad, f"kernels with scratch or spills in {os.path.basename(obj)}: {bad}"
