"""Host logic of the fused DAgger path (CPU): which adaptation-encoder shapes lgx_adaptation_train's
tiling covers (hip_mlp.adaptation_train_supported mirrors the checks of the C entry point), and the
grid / chunk arithmetic the per-block gradient rows are sized by."""
import torch

from legged_gym_custom_amd.rsl_rl.modules import hip_mlp as H
from legged_gym_custom_amd.rsl_rl.modules.support_networks import AdaptationEncoder


def test_go2_encoder_is_covered():
    mod = AdaptationEncoder(num_proprio=52, history_buffer_length=10)
    assert H.adaptation_train_supported(mod, 52)


def test_shapes_outside_the_tiling_fall_back():
    # a long history: the first convolution leaves more than 4 positions (weight-gradient K slots)
    assert not H.adaptation_train_supported(AdaptationEncoder(num_proprio=52, history_buffer_length=20), 52)
    # a wide proprio vector: the fc_encoder fragment exceeds 16 K steps in registers
    assert not H.adaptation_train_supported(AdaptationEncoder(num_proprio=72, history_buffer_length=10), 72)


def test_grid_covers_every_row_once():
    for rows in (1, 15, 16, 17, 4805, 24576, 49152):
        for blocks in (1, 7, 512, 768):
            grid = H.adapt_train_grid(rows, blocks)
            nchunk = -(-rows // H.ADAPT_TRAIN_ROWS)
            chunks = -(-nchunk // blocks)
            assert grid <= blocks and grid * chunks >= nchunk and (grid - 1) * chunks < nchunk
