"""Stage block-shape choice (ops/hip_compute.choose_block), CPU only."""
from stsphere.ops.hip_compute import BLOCK_SHAPES, block_supports, choose_block


def test_full_c96_grid_keeps_16x16():
    assert choose_block(48, 24, 256, 2) == (16, 16)      # 216 blocks: one pass over 256 CUs


def test_small_rank_grids_take_smaller_blocks():
    # profiles/r1_small_grid_block_shapes.txt: 12 tiles -> 16x8, 6 / 3 tiles -> 8x8
    assert choose_block(48, 12, 256, 2) == (16, 8)
    assert choose_block(48, 6, 256, 2) == (8, 8)
    assert choose_block(48, 3, 256, 2) == (8, 8)


def test_multi_pass_grids_take_small_blocks():
    # profiles/r1_block_shapes_by_size.txt: several blocks per CU -> 16x8 (fp32,
    # mid-size fp64), 8x8 for large fp64 grids; PPM never gets 8x8
    assert choose_block(64, 24, 256, 2, esize=4) == (16, 8)      # C128 fp32
    assert choose_block(90, 24, 256, 2, esize=8) == (16, 8)      # C180 fp64
    assert choose_block(128, 24, 256, 2, esize=8) == (8, 8)      # C256 fp64
    assert choose_block(360, 24, 256, 2, esize=8) == (8, 8)      # C720 fp64
    assert choose_block(360, 24, 256, 2, esize=4) == (16, 8)     # C720 fp32
    assert choose_block(360, 24, 256, 4, esize=8) == (16, 8)     # PPM


def test_ppm_never_gets_a_block_too_small_for_its_window():
    assert not block_supports(8, 8, 4) and block_supports(16, 8, 4)
    for n, t in ((48, 3), (48, 6), (12, 24), (24, 6)):
        bx, by = choose_block(n, t, 256, 4)
        assert block_supports(bx, by, 4) and (bx, by) in BLOCK_SHAPES


def test_without_device_info_falls_back_to_least_waste():
    assert choose_block(48) == (16, 16)
    assert choose_block(40) in ((16, 16), (32, 8))


def test_fused_block_by_rank_share():
    """ops/fused.py::fused_block: the smallest fused block whose blocks are all
    resident on the rank's CUs.  C96 (24 tiles of 48) on 1 / 2 / 4 / 8 GPUs of
    256 CUs: B = 16 (216 blocks), 12 (192), 8 (216), 6 (192,
    profiles/r5_rehearse/b6); a shared-GPU rehearsal counts its share of the
    CUs; a grid whose blocks never all fit takes the largest block."""
    from stsphere.ops.fused import fused_block
    assert [fused_block(48, 24 // r, 256) for r in (1, 2, 4, 8)] == [16, 12, 8, 6]
    assert fused_block(48, 3, 32) == 16                  # 8 ranks sharing one GPU
    assert fused_block(90, 24, 256) == 18                # C180 on one GPU: never resident
    assert fused_block(96, 1, 256) == 6                  # one panel per rank (6 GPUs): 256 blocks
    assert fused_block(14, 6, 256) is None
