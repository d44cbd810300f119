"""GEMM launch plans (CPU: pure shape arithmetic in kubeflow_rm_amd.ops.gemm)."""
from kubeflow_rm_amd.ops import gemm


def test_fixk_plan_takes_few_tile_problems():
    # 4096x2048x8192: 128 tiles of 256 -> two K-splits fill the 256 CUs, 64 K-tiles each
    assert gemm.fixk_plan(4096, 2048, 8192) == (2, 4096)
    # a deep-K gpt-small weight gradient: 36 tiles, 7 splits
    splits, kper = gemm.fixk_plan(3072, 768, 32768)
    assert splits == 7 and kper % 64 == 0 and (splits - 1) * kper < 32768 <= splits * kper
    assert 36 * splits <= gemm._NUM_CUS
    # a square projection's weight gradient, 64 tiles: four splits of 32 K-tiles
    assert gemm.fixk_plan(2048, 2048, 8192) == (4, 2048)
    # 32 K-tiles in all: nothing to split
    assert gemm.fixk_plan(2048, 2048, 2048) is None
    # enough tiles to fill the chip, or too few for the 256 tile: other paths
    assert gemm.fixk_plan(8192, 8192, 8192) is None
    assert gemm.fixk_plan(6144, 2048, 8192) is None
    assert gemm.fixk_plan(768, 768, 32768) is None  # 9 tiles: the 128-tile split-K
    # shallow K: nothing to split
    assert gemm.fixk_plan(2048, 2048, 1024) is None
    # off the 8-element grid / below the tile
    assert gemm.fixk_plan(2048, 2046, 8192) is None
    assert gemm.fixk_plan(200, 4096, 8192) is None


def test_fixk_plan_switches():
    old = gemm.FIXK
    try:
        gemm.FIXK = False
        assert gemm.fixk_plan(2048, 2048, 8192) is None
    finally:
        gemm.FIXK = old
    gemm.FIXK_SPLITS = 3
    try:
        assert gemm.fixk_plan(8192, 8192, 8192) == (3, 2752)
    finally:
        gemm.FIXK_SPLITS = None
