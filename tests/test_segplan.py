"""Segment-launch geometry on the host (CPU): tests/cxx/segplan_check.cpp, built with hipcc, walks the
product's segment tables (vd_segplan.h) through the kernel's own segment functions (vd_kernel_tg.h
seg_bound / seg_run) for the bench sizes and random chunk lengths: every word of every chunk is emitted by
exactly one segment, speculative starts are group-aligned and always meet a left neighbour's end vector
at the same block, no segment is empty.  The GPU tests then check the decoded words."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_segment_geometry(tmp_path):
    exe = tmp_path / "segplan_check"
    src = os.path.join(ROOT, "tests", "cxx", "segplan_check.cpp")
    csrc = os.path.join(ROOT, "gpu-accelerated-viterbi-decoder_amd", "csrc")
    r = subprocess.run([HIPCC, "-x", "hip", "--offload-arch=gfx950", "-O1", "-std=c++17", "-w", "-I", csrc, src,
                        "-o", str(exe)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stdout[-2000:]
