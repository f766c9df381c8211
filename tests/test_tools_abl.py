"""The product kernel headers carry no ablation code; tools/abl/gen_abl.py re-inserts the tools-only ablation
bits (ABL) into copies under tools/build/abl, and those copies still compile for gfx950 (the timing tools
include them).  CPU only: a device-only compile of a few ablation instantiations."""
import os
import re
import subprocess
import sys
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "gpu-accelerated-viterbi-decoder_amd", "csrc")
sys.path.insert(0, os.path.join(ROOT, "tools", "abl"))
import gen_abl  # noqa: E402


def test_product_headers_have_no_ablation_code():
    for name in os.listdir(CSRC):
        if name.endswith((".h", ".hip", ".cpp")):
            text = open(os.path.join(CSRC, name)).read()
            assert not re.search(r"\bABL\b|kAbl", text), name


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="hipcc not available")
def test_generated_ablation_headers_compile():
    with tempfile.TemporaryDirectory() as d:
        gen_abl.main(os.path.join(d, "abl"))
        tu = os.path.join(d, "tu.hip")
        with open(tu, "w") as f:
            f.write('#include "abl/vd_kernel_pk.h"\n'
                    "template __global__ void vd::vd_decode_pk<vd::SOFT8, vd::B16, 32, false, 7, vd::kAblAcsOnly>"
                    "(const void*, void*, vd::Geom);\n"
                    "template __global__ void vd::vd_decode_pk<vd::HARD, vd::B32, 32, true, 7, vd::kAblClock | vd::kAblNoStores>"
                    "(const void*, void*, vd::Geom);\n"
                    "template __global__ void vd::vd_decode_tg<vd::SOFT16, vd::B32, 32, vd::kAblNoTraceback | vd::kAblClock>"
                    "(const void*, void*, vd::Geom);\n")
        r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", "-c",
                            "-I", d, "-I", CSRC, tu, "-o", os.path.join(d, "tu.o")], capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stderr[-3000:]
