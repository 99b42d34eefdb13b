"""GPU parity of the feature frontend (csrc/fbank.hip, statecatcher_amd.frontend) — SURVEY §8(f)
row 3 — against oracle/fbank.py (fp64 numpy restatement of torchaudio's MFCC / MelSpectrogram +
AmplitudeToDB with make_frontend's arguments, model.py:250-279), itself pinned by
tests/golden/fbank.npz (transformers audio_utils + scipy DCT).  fp32 kernel: MFCC within
1e-3 of the coefficient scale, log-mel within 1e-3 dB."""
import numpy as np
import pytest
import torch

from oracle import fbank as ofb
from tests.conftest import load_golden

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0") if torch.cuda.is_available() else None


def ops():
    from statecatcher_amd import ops as o
    return o


def close(got, ref, frac=1e-3):
    got = got.detach().double().cpu().numpy()
    np.testing.assert_allclose(got, ref, rtol=frac, atol=frac * max(np.abs(ref).max(), 1.0))


@pytest.mark.parametrize("kind,key", [("mfcc", "mfcc"), ("mel", "logmel_db")])
def test_fbank_vs_fixture(kind, key):
    z = load_golden("fbank")
    out = ops().fbank(torch.as_tensor(z["audio"]).to(DEV), kind)
    assert out.shape == z[key].shape
    close(out, z[key])


@pytest.mark.parametrize("kind", ["mfcc", "mel"])
def test_fbank_vs_oracle_long_and_strided(kind):
    """3 s rows of speech-like noise at 16 kHz (298 frames), one silent row, a row-strided
    view (an audio buffer with padding between rows), and the frame-count edge cases."""
    g = torch.Generator().manual_seed(3)
    B, N = 4, 48000
    buf = torch.randn(B, N + 37, generator=g) * 0.3
    buf[2] = 0.0
    t = torch.arange(N + 37) / 16000.0
    buf[1] += 0.5 * torch.sin(2 * np.pi * 1000.0 * t)
    audio = buf[:, :N]                                  # row stride N + 37
    out = ops().fbank(buf.to(DEV)[:, :N], kind)
    ref = ofb.frontend(audio.numpy(), kind)
    assert out.shape == ref.shape == (B, 298, 80)
    close(out, ref)
    for n, frames in ((399, 0), (400, 1), (559, 1), (560, 2)):
        o = ops().fbank(buf[:2, :n].contiguous().to(DEV), kind)
        assert o.shape == (2, frames, 80)
        if frames:
            close(o, ofb.frontend(buf[:2, :n].numpy(), kind))


def test_make_frontend_module_shapes_and_topdb_packing():
    """make_frontend returns (module, mel kwargs) as model.py:250-279; the module maps [..., time]
    to [..., 80, frames]; log-mel's top_db floor follows AmplitudeToDB's dim -3 packing: batch-
    wide for [B, time] audio, per leading item for [B, C, time]."""
    import statecatcher_amd as sc
    fe, kw = sc.make_frontend("mfcc", 16000)
    assert kw["n_fft"] == 400 and kw["hop_length"] == 160 and kw["mel_scale"] == "htk"
    g = torch.Generator().manual_seed(4)
    a = torch.randn(2, 16000, generator=g)
    y = fe(a.to(DEV))
    assert y.shape == (2, 80, 98)
    close(y.transpose(1, 2), ofb.frontend(a.numpy(), "mfcc"))
    assert fe(a[0].to(DEV)).shape == (80, 98)
    with pytest.raises(ValueError):
        sc.make_frontend("plp", 16000)
    mel, _ = sc.make_frontend("mel", 16000)
    loud = torch.cat([a[:1] * 1000.0, a[1:] * 1e-3])       # 120 dB apart
    y2 = mel(loud.to(DEV)).transpose(1, 2)
    close(y2, ofb.frontend(loud.numpy(), "mel"))            # one batch-wide floor
    y3 = mel(loud[:, None, :].to(DEV))                      # [B, 1, time]: per-item floors
    assert y3.shape == (2, 1, 80, 98)
    close(y3[1, 0].transpose(0, 1), ofb.frontend(loud[1:].numpy(), "mel")[0])
