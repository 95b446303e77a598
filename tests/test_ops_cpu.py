"""torch.ops.m2s.* on CPU: libm2s_torch.so loads, registers every op, and the fake (meta) kernels
give the shapes the HIP kernels produce (FakeTensor tracing / torch.compile).  No GPU needed."""
import pytest
import torch

from m2s import ops


@pytest.fixture(scope="module")
def m2s_ops():
    return ops.load()


def test_every_op_registered(m2s_ops):
    for name in ops.OPS:
        assert hasattr(m2s_ops, name), name
        assert str(getattr(torch.ops.m2s, name).default._schema).startswith(f"m2s::{name}(")


def test_fake_shapes(m2s_ops):
    meta = lambda *s: torch.empty(*s, device="meta")  # noqa: E731
    assert m2s_ops.acoustic_forward(1, meta(2, 30, 256, 256), 64).shape == (2, 30, 64)
    assert m2s_ops.effnet_forward(1, meta(7, 256, 256)).shape == (7, 208)
    y, m = m2s_ops.bilstm_summerge(1, meta(3, 9, 208), 640, 64)
    assert y.shape == (3, 9, 640) and m.shape == (3, 9, 64)
    db, ln = m2s_ops.mel_glue(meta(5, 64), meta(64), meta(64))
    assert db.shape == ln.shape == (5, 64)
    assert m2s_ops.hifigan_forward(2, meta(2, 64, 30), 0, 420).shape == (2, 1, 12600)
    assert m2s_ops.hifigan_forward(2, meta(2, 30, 64), 1, 420).shape == (2, 1, 12600)
    outs = m2s_ops.pipeline_forward(1, 2, meta(4, 30, 256, 256), meta(64), meta(64), 64, 420)
    assert [tuple(t.shape) for t in outs] == [(4, 30, 64)] * 3 + [(4, 12600)]
    assert m2s_ops.preprocess_frames(torch.empty(3, 64, 48, 3, dtype=torch.uint8, device="meta")).shape == (3, 64, 48)


@pytest.mark.parametrize("hw,n,shape", [((256, 256), 0, (32, 128, 128)), ((256, 256), 2, (16, 128, 128)),
                                        ((256, 256), 5, (32, 64, 64)), ((256, 256), 8, (56, 32, 32)),
                                        ((256, 256), 18, (120, 16, 16)), ((256, 256), 28, (208, 8, 8)),
                                        ((67, 101), 28, (208, 3, 4))])
def test_feature_shapes_follow_tf_same(m2s_ops, hw, n, shape):
    got = m2s_ops.effnet_features(1, torch.empty(2, *hw, device="meta"), n)
    assert tuple(got.shape) == (2,) + shape
