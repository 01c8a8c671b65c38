"""Register budget of the conv-1 forward (CPU: hipcc cross-compiles gfx950 here).

The split-f16 row-GEMM forward (csrc/conv_rows.h) runs two 512-thread workgroups per CU only while
it needs <= 128 VGPRs: one more register halves its occupancy, and the catalogue conv-1 forward --
the largest launch of a catalogue step -- went 92 -> 120 us when a slab-fill change took it to 156
(round 3). This compiles conv_fwd.hip with the kernel-resource remarks and holds every non-DEEP
split-f16 conv-1 instance (the ones launched with several workgroups per CU) to 128 VGPRs and no
scratch.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "amplifai-deepcontentrecommenders_amd")
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_conv1_forward_fits_two_workgroups_per_cu(tmp_path):
    out = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                          "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(PKG, "csrc"), "-c",
                          os.path.join(PKG, "csrc", "conv_fwd.hip"), "-o", str(tmp_path / "conv_fwd.o"),
                          "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    res, cur = {}, None
    for line in out.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            res[cur] = {}
            continue
        m = re.search(r"(VGPRs|ScratchSize \[bytes/lane\]): (\d+)", line)
        if m and cur:
            res[cur][m.group(1).split(" ")[0]] = int(m.group(2))
    # k_conv_rows<MODE 0, SRC_TRACK_F16 (0), KC 128, ..., DEEP false, F16 true>
    conv1 = {k: v for k, v in res.items() if "k_conv_rowsILi0ELi0ELi128E" in k and k.endswith("Lb0ELb1EEEvNS_8RowsArgsE")}
    assert conv1, "no split-f16 conv-1 forward instance found"
    for k, v in conv1.items():
        assert v.get("VGPRs", 999) <= 128 and v.get("ScratchSize", 0) == 0, (k, v)
