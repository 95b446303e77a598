"""Grad-CAM path on the GPU vs torch-CPU autograd over the oracle.

The caller below drives the plug-in exactly the way the reference's scripts/mri_gradcam_formant.py
does (compute_gradcam :203-279 with _forward_with_features :128-166 and _compute_cam_from_grads
:169-200): model.train() with the rnn dropout in eval, backbone of the RGB-repeated frames, last map
made a gradient leaf, mean -> rnn -> head, band power of the de-normalised mel, backward, feats.grad.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from m2s import synth
from oracle import acoustic, effnet, gradcam

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _t(sd):
    return {k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()}


def _model(seed):
    from mri_acoustic_model import build_acoustic_model
    m = build_acoustic_model(n_mels=64, cnn_pretrained=False, rnn_hidden=640, dropout=0.5).to(DEV)
    m.load_state_dict(_t(synth.synth_acoustic_state(seed)), strict=False)
    return m.eval()


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


# --- the caller (the reference script's sequence of module calls) ---------------------------------
def _cam(feats, grads, B, T, hw):
    w = grads.mean(dim=(2, 3), keepdim=True)
    cam = torch.relu((w * feats).sum(dim=1, keepdim=True)).view(B, T, *feats.shape[-2:]).detach()
    out = []
    for t in range(T):
        c = F.interpolate(cam[:, t].unsqueeze(1), size=hw, mode="bilinear", align_corners=False).squeeze(1)
        c = c - c.amin(dim=(-2, -1), keepdim=True)
        out.append(c / (c.amax(dim=(-2, -1), keepdim=True) + 1e-6))
    return torch.stack(out, dim=1).squeeze(0)


def run_gradcam(model, frames, mean, std, band, reduction="mean", frame_indices=()):
    was_training, drop_state = model.training, model.rnn.dropout.training
    model.train()
    model.rnn.dropout.train(False)
    B, T = frames.shape[:2]
    x = frames.reshape(B * T, *frames.shape[2:]).repeat(1, 3, 1, 1)
    feats = model.cnn.backbone(x)[-1]
    feats = feats.requires_grad_(True)
    feats.retain_grad()
    pred = model.head(model.rnn(feats.mean(dim=(2, 3)).view(B, T, -1)))
    power = torch.pow(10.0, (pred * torch.from_numpy(std).to(DEV) + torch.from_numpy(mean).to(DEV)) / 10.0)
    band_power = power.index_select(-1, torch.as_tensor(list(band), device=DEV)).sum(-1)
    frames_l = list(frame_indices)
    model.zero_grad(set_to_none=True)
    (band_power.mean() if reduction == "mean" else band_power.sum()).backward(retain_graph=bool(frames_l))
    grads = feats.grad.detach().clone()
    maps = _cam(feats.detach(), grads, B, T, tuple(frames.shape[-2:]))
    per = {}
    for i, t in enumerate(frames_l):
        model.zero_grad(set_to_none=True)
        feats.grad.zero_()
        band_power[:, t].mean().backward(retain_graph=i < len(frames_l) - 1)
        per[t] = _cam(feats.detach(), feats.grad.detach().clone(), B, T, tuple(frames.shape[-2:]))[t]
    model.rnn.dropout.train(drop_state)
    if not was_training:
        model.eval()
    return maps, per, grads


# --- pieces ---------------------------------------------------------------------------------------
def test_train_mode_backbone_uses_batch_statistics():
    """model.train(): every feature map from batch-statistics BatchNorm (timm / torch train mode) and
    the running statistics updated like torch's (momentum 0.1, unbiased variance), vs the oracle."""
    m = _model(3).train()
    fr = synth.synth_frames(1, 5, seed=21)[0]
    x = torch.from_numpy(fr)[:, None]
    with torch.no_grad():
        maps = m.cnn.backbone(x.to(DEV).repeat(1, 3, 1, 1))
    sd = _t(synth.synth_acoustic_state(3))
    taps = []
    effnet.effnet_features(sd, x, taps=taps, train=True)
    for got, k in zip(maps, (2, 5, 8, 18, 28)):
        assert tuple(got.shape) == tuple(taps[k].shape)
        assert _rel(got.cpu(), taps[k]) < 1e-4, k
    msd = m.state_dict()
    for key in ("cnn.backbone.bn1", "cnn.backbone.blocks.1.0.bn2", "cnn.backbone.blocks.5.9.bn3"):
        for b in ("running_mean", "running_var"):
            assert _rel(msd[f"{key}.{b}"].cpu(), sd[f"{key}.{b}"]) < 1e-4, (key, b)
        assert int(msd[f"{key}.num_batches_tracked"]) == 1
    # eval afterwards uses the updated running statistics (the inference engine repacks)
    m.eval()
    with torch.no_grad():
        f_eval = m.cnn(x.to(DEV)).cpu()
    ref = effnet.effnet_gap(sd, x)
    assert _rel(f_eval, ref) < 1e-3


@pytest.mark.parametrize("B,T", [(1, 9), (3, 5)])
def test_bilstm_autograd_matches_torch(B, T):
    """model.rnn with autograd: output, dx and every nn.LSTM weight gradient vs torch-CPU autograd."""
    m = _model(5).train()
    m.rnn.dropout.train(False)
    g = torch.Generator().manual_seed(B * 100 + T)
    x = torch.randn(B, T, 208, generator=g)
    wy = torch.randn(B, T, 640, generator=g)
    xd = x.to(DEV).requires_grad_(True)
    y = m.rnn(xd)
    (y * wy.to(DEV)).sum().backward()
    ref_lstm = torch.nn.LSTM(208, 640, 1, batch_first=True, bidirectional=True)
    ref_lstm.load_state_dict({k[len("rnn.lstm."):]: v for k, v in _t(synth.synth_acoustic_state(5)).items()
                              if k.startswith("rnn.lstm.")})
    xr = x.clone().requires_grad_(True)
    yr = ref_lstm(xr)[0]
    yr = yr[..., :640] + yr[..., 640:]
    (yr * wy).sum().backward()
    assert _rel(y.detach().cpu(), yr.detach()) < 1e-5
    assert _rel(xd.grad.cpu(), xr.grad) < 1e-5
    for name, p in ref_lstm.named_parameters():
        got = getattr(m.rnn.lstm, name).grad
        assert got is not None, name
        assert _rel(got.cpu(), p.grad) < 1e-5, name


def test_head_and_gap_autograd():
    m = _model(6)
    g = torch.Generator().manual_seed(4)
    x = torch.randn(2, 7, 640, generator=g)
    xd = x.to(DEV).requires_grad_(True)
    y = m.head(xd)
    w = torch.randn(2, 7, 64, generator=g)
    (y * w.to(DEV)).sum().backward()
    lin = torch.nn.Linear(640, 64)
    lin.load_state_dict({"weight": m.head.weight.detach().cpu(), "bias": m.head.bias.detach().cpu()})
    xr = x.clone().requires_grad_(True)
    (lin(xr) * w).sum().backward()
    assert _rel(y.detach().cpu(), lin(x).detach()) < 1e-5
    assert _rel(xd.grad.cpu(), xr.grad) < 1e-5
    assert _rel(m.head.weight.grad.cpu(), lin.weight.grad) < 1e-5
    assert _rel(m.head.bias.grad.cpu(), lin.bias.grad) < 1e-5
    f = torch.randn(3, 208, 8, 8, generator=g)
    fd = f.to(DEV).requires_grad_(True)
    p = m.cnn.gap(fd)
    wp = torch.randn(3, 208, generator=g)
    (p * wp.to(DEV)).sum().backward()
    fr = f.clone().requires_grad_(True)
    (fr.mean(dim=(2, 3)) * wp).sum().backward()
    assert _rel(p.detach().cpu(), f.mean(dim=(2, 3))) < 1e-6
    assert _rel(fd.grad.cpu(), fr.grad) < 1e-6


# --- end to end -----------------------------------------------------------------------------------
@pytest.mark.parametrize("reduction", ["mean", "sum"])
def test_gradcam_matches_oracle(reduction):
    """Heat maps (full target and per-frame targets) within 1e-4 of torch-CPU autograd over the
    oracle; feats.grad within 1e-4 relative."""
    m = _model(3)
    mean, std = synth.synth_scaler()
    fr = torch.from_numpy(synth.synth_frames(1, 6, seed=11))[:, :, None]
    band = list(range(5, 20))
    maps, per, grads = run_gradcam(m, fr.to(DEV), mean, std, band, reduction, [0, 5])
    assert not m.training and not m.rnn.dropout.training
    rmaps, rper, rgrads = gradcam.gradcam(_t(synth.synth_acoustic_state(3)), fr, mean, std, band, reduction, [0, 5])
    assert _rel(grads.cpu(), rgrads) < 1e-4
    assert tuple(maps.shape) == (6, 256, 256)
    np.testing.assert_allclose(maps.cpu().numpy(), rmaps.numpy(), atol=1e-4, rtol=0)
    for t in (0, 5):
        np.testing.assert_allclose(per[t].cpu().numpy(), rper[t].numpy(), atol=1e-4, rtol=0)


def test_train_mode_forward_no_grad_and_cnn_backward_refused():
    """model(x) in train() under no_grad = batch-statistics backbone -> GAP -> rnn -> head (the
    reference's training-mode graph, mri_acoustic_model.py:116-130); with gradients enabled it refuses
    (no backbone backward) instead of returning gradient-less outputs."""
    m = _model(4).train()
    m.rnn.dropout.train(False)  # Dropout(0.5) is live in train(): compare the deterministic graph
    fr = synth.synth_frames(1, 4, seed=8)
    x = torch.from_numpy(fr)[:, :, None]
    with torch.no_grad():
        out = m(x.to(DEV)).cpu()
    sd = _t(synth.synth_acoustic_state(4))
    feats = effnet.effnet_features(sd, x[0], train=True).mean(dim=(2, 3)).view(1, 4, -1)
    ref = acoustic.head(sd, acoustic.bilstm_summerge(sd, feats))
    assert _rel(out, ref) < 1e-4
    with pytest.raises(NotImplementedError):
        m(x.to(DEV))
