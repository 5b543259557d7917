"""The codebook-pinned VQ forward's LDS images (csrc/vq.hip, vq_pos): dims permuted even-then-odd so that MFMA lane
half h reads four consecutive 32x32x2 steps as one 16-B read, and 16-B quads XOR-swizzled by the row.  CPU-only
restatement of the address map: every position of a row is used once, the four steps a lane reads are its dims in
k order, and the operand reads of a ds_read_b128 lane group hit 16 distinct bank slots at D = 64."""
import os

import pytest

SRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "vq-vae-transformer-arc-welding_amd",
                   "csrc", "vq.hip")

B128_GROUPS = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
               list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
B128_GROUPS += [[lane + 32 for lane in g] for g in B128_GROUPS]


def test_restatement_matches_the_kernel_source():
    text = open(SRC).read()
    assert "return c * D + ((((p >> 2) ^ c) & (D / 4 - 1)) << 2) + (p & 3);" in text
    assert "*reinterpret_cast<float2*>(img + vq_pos<D>(c, 2 * q)) = make_float2(v.x, v.z);" in text
    assert "*reinterpret_cast<float2*>(img + vq_pos<D>(c, H2 + 2 * q)) = make_float2(v.y, v.w);" in text


def vq_pos(D, c, p):
    """float offset of permuted position p of row c (the kernel's vq_pos)"""
    return c * D + ((((p >> 2) ^ c) & (D // 4 - 1)) << 2) + (p & 3)


def perm(D, d):
    """permuted position of dim d: even dims first, then odd"""
    return (d & 1) * (D // 2) + (d >> 1)


@pytest.mark.parametrize("D", [16, 32, 64])
def test_positions_are_a_permutation_of_each_row(D):
    for c in range(40):
        offs = sorted(vq_pos(D, c, perm(D, d)) for d in range(D))
        assert offs == list(range(c * D, c * D + D))


@pytest.mark.parametrize("D", [16, 32, 64])
def test_a_lane_reads_its_steps_in_k_order(D):
    # lane half h reads steps s .. s + 3 (dims 2s + h, 2s + 2 + h, ...) as one float4 at permuted position h D/2 + s
    for c in range(8):
        for h in range(2):
            for s in range(0, D // 2, 4):
                base = vq_pos(D, c, h * (D // 2) + s)
                assert base % 4 == 0
                for i in range(4):
                    assert vq_pos(D, c, perm(D, 2 * (s + i) + h)) == base + i


def test_operand_reads_are_conflict_free_at_d64():
    D = 64
    for row_base in (0, 32, 64, 448):          # code tiles of different waves, z row tiles
        for s in range(0, D // 2, 4):
            for grp in B128_GROUPS:
                slots = {(vq_pos(D, row_base + (lane & 31), (lane >> 5) * (D // 2) + s) // 4) % 16 for lane in grp}
                assert len(slots) == 16, (row_base, s, grp)
