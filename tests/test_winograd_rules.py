"""Host-side Winograd dispatch rules (ops._wino_ok / _wino_blocks / _wino_alg): no GPU needed."""
import pytest

from medvae_disentangled_multimodal_amd import ops

G3 = ops.ConvGeom(3, 3, 1, 1, 1, 1, 1, False)


@pytest.fixture
def rules(monkeypatch):
    monkeypatch.setattr(ops, "WINOGRAD", True)
    monkeypatch.setattr(ops, "WINOGRAD_TILE", 4)
    monkeypatch.setattr(ops, "WINOGRAD_MAX_W", 64)
    monkeypatch.setattr(ops, "WINOGRAD_MIN_C", 512)
    monkeypatch.setattr(ops, "WINOGRAD_MIN_C_WIDE", 256)
    monkeypatch.setattr(ops, "WINOGRAD_MIN_MACS", 1e10)
    monkeypatch.setattr(ops, "_MATH", [0])  # (a private list: the process-wide mode is untouched)
    return monkeypatch


def test_c4_levels(rules):
    """c4 at B = 256: every 3x3 / stride-1 level runs Winograd (the 64x64 level at 256 channels: images >= 32 wide take
    >= 256 channels), except the 64x64 conv with a 512-channel side (operand over 4 GiB); non-3x3 / strided /
    upsample convs the implicit GEMM."""
    assert ops._wino_ok(G3, 256, 8, 8, 2048, 2048)
    assert ops._wino_ok(G3, 256, 16, 16, 1024, 1024)
    assert ops._wino_ok(G3, 256, 32, 32, 512, 512)
    assert ops._wino_ok(G3, 256, 32, 32, 1024, 512)
    assert ops._wino_ok(G3, 256, 64, 64, 256, 256)
    assert ops._wino_ok(G3, 256, 64, 64, 512, 256)            # 36 x 65,536 x 512 x 4 B > 4 GiB: two image chunks
    assert not ops._wino_ok(G3, 256, 32, 32, 128, 512)        # 128 input channels
    assert not ops._wino_ok(G3, 256, 14, 14, 256, 256)        # narrow images need 512 channels
    assert not ops._wino_ok(G3, 64, 128, 128, 256, 256)       # width above MAX_W
    assert not ops._wino_ok(ops.ConvGeom(1, 1), 256, 16, 16, 1024, 1024)
    assert not ops._wino_ok(ops.ConvGeom(3, 3, 2, 0, 0, 1, 1), 256, 16, 16, 512, 512)
    assert not ops._wino_ok(ops.ConvGeom(3, 3, 1, 1, 1, 1, 1, True), 256, 16, 16, 512, 512)


def test_small_batches_and_math_modes(rules):
    assert ops._wino_ok(G3, 256, 7, 7, 512, 512)              # c2's 7x7 level (29.6 GMAC)
    assert not ops._wino_ok(G3, 32, 7, 7, 512, 512)           # c1 at B = 32 (3.7 GMAC): below MIN_MACS
    rules.setattr(ops, "WINOGRAD_TILE_BF16", 2)
    rules.setattr(ops, "WINOGRAD_BF16_MAX_W", 16)
    ops._MATH[0] = 1                                          # bf16-mixed (c5): F(2x2) at the small wide levels only
    assert ops._wtile() == 2 and ops._wino_alg(36.0) == pytest.approx(16.0)
    assert ops._wino_ok(G3, 256, 8, 8, 2048, 2048) and ops._wino_ok(G3, 256, 16, 16, 1024, 1024)
    assert not ops._wino_ok(G3, 256, 32, 32, 512, 512) and not ops._wino_ok(G3, 256, 64, 64, 256, 256)
    assert ops._wino_chunks(256, 16, 16, 1024) == [(0, 256)]  # (F2: 16 x 16,384 tiles x 1024 x 4 B = 1.07 GB)
    rules.setattr(ops, "WINOGRAD_BF16", False)
    assert not ops._wino_ok(G3, 256, 8, 8, 2048, 2048)
    ops._MATH[0] = 2                                          # exact fp32 (c4x): F(4x4) at every c4 level
    assert ops._wtile() == 4
    assert ops._wino_ok(G3, 256, 8, 8, 2048, 2048) and ops._wino_ok(G3, 256, 64, 64, 512, 256)
    rules.setattr(ops, "WINOGRAD_EXACT", False)
    assert not ops._wino_ok(G3, 256, 8, 8, 2048, 2048)


def test_size_rule_chunks_operands_under_4gib(rules):
    """Transformed operands over one 4 GiB buffer descriptor run in image chunks (the 64x64x512 decoder conv at B = 256:
    36 x 65,536 tiles x 512 channels x 4 B = 4.8 GB -> two halves); more than WINOGRAD_MAX_CHUNKS chunks stay on the
    implicit GEMM."""
    assert ops._wino_chunks(256, 64, 64, 256) == [(0, 256)]
    chunks = ops._wino_chunks(256, 64, 64, 512)
    assert len(chunks) == 2 and chunks[0][0] == 0 and chunks[-1][1] == 256
    assert all(36 * ops._wino_tiles(b1 - b0, 64, 64) * 512 * 4 <= ops._MAX_DESC_BYTES for b0, b1 in chunks)
    assert ops._wino_ok(G3, 1024, 32, 32, 512, 512)           # c4's 32x32 level at B = 1024: 2 chunks
    assert not ops._wino_ok(G3, 2048, 64, 64, 512, 256)       # 10 chunks


def test_block_geometry_and_flop_accounting(rules):
    assert ops._wino_blocks(8, 8) and ops._wino_blocks(16, 16) and ops._wino_blocks(32, 32) and ops._wino_blocks(4, 64)
    assert not ops._wino_blocks(7, 7) and not ops._wino_blocks(14, 14) and not ops._wino_blocks(6, 8)
    assert ops._wino_alg(36.0) == pytest.approx(9.0)           # F(4x4, 3x3): 36 / 144 of the direct MACs
    rules.setattr(ops, "WINOGRAD_TILE", 2)
    assert ops._wino_alg(36.0) == pytest.approx(16.0)          # F(2x2, 3x3): 16 / 36
    assert ops._wino_tiles(3, 7, 7) == 3 * 4 * 4               # edge tiles counted
