"""Host model of the packed split kernel's pass loop (tools/split_model.py): the re-decode passes end within P
(P = 2 parts per whole-chunk wave, 8 per tail workgroup), so the kernel's cap of 2 P passes never binds and
vd_split_cap_exits stays 0; every part's start and end vectors equal one decode of the whole chunk, on
random bytes, noisy codewords and a chunk that never forgets its start vector (exactly P passes)."""
import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import split_model as sm  # noqa: E402


@pytest.mark.parametrize("P,W", [(2, 64), (2, 157), (8, 157)])
@pytest.mark.parametrize("kind", ["random", "codeword", "no-convergence"])
@pytest.mark.parametrize("warm", [sm.K_WARM, 0])
def test_split_passes_end_within_P(P, W, kind, warm):
    passes = [sm.check(W, P, kind, seed, warm) for seed in range(3)]
    assert max(passes) <= P < 2 * P
    if kind == "no-convergence":
        assert passes == [P] * 3  # the bound is reached: the model is not vacuous
    if kind == "random" and warm == 0:
        assert max(passes) >= 2  # starts from equal metrics fail on noise: re-decodes ran


def test_pk_cut_matches_the_kernel():
    """pk_cut as vd_kernel_pk.h computes it: part origins minus the warm-up are multiples of 3 blocks"""
    for W in (64, 78, 157, 300):
        for P in (2, 8):
            cuts = [sm.pk_cut(p, P, W) for p in range(P + 1)]
            assert cuts[0] == 0 and cuts[-1] == W and cuts == sorted(cuts)
            assert all((c - sm.K_WARM) % 3 == 0 for c in cuts[1:-1])
