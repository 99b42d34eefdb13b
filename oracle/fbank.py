"""Feature frontend oracle (TEST INFRASTRUCTURE ONLY): the reference's `make_frontend`
(model.py:250-279), applied under no_grad at train.py:473-475, restated in numpy fp64.

The reference builds it from torchaudio (unpinned; not in requirements.txt, absent from this
container and from /root/reference), so parity w.r.t. torchaudio itself is UNPINNED.  This file
restates the published torchaudio algorithms the two frontends chain, with the reference's
arguments (n_fft = win_length = 400, hop_length = 160, n_mels = 80, center=False, power=2.0,
mel_scale="htk", sample rate 16 kHz):

  spectrogram     torchaudio.functional.spectrogram: frames x[f*hop : f*hop + n_fft] (no
                  centring / padding), times torch.hann_window(400) (periodic), one-sided DFT
                  (np.fft.rfft here), |X|^2 (power 2, normalized=False)
  melscale_fbanks torchaudio.functional.melscale_fbanks(n_freqs=201, f_min=0, f_max=sr/2,
                  n_mels=80, sample_rate, norm=None, mel_scale="htk"): triangular filters
                  between n_mels+2 points equally spaced in HTK mel, mel = 2595 log10(1 + f/700)
  MFCC ("mfcc")   log(mel + 1e-6) (log_mels=True), then the DCT-II matrix of create_dct(n_mfcc=80,
                  n_mels=80, norm="ortho")
  log-mel ("mel") AmplitudeToDB(stype="power", top_db=80): 10 log10(max(x, 1e-10)) (ref 1.0,
                  amin 1e-10), then max(x_db, max - 80) where, for a 3-D (B, n_mels, frames)
                  input, the max runs over the whole tensor (amplitude_to_DB packs dim -3)

Output layout (B, frames, 80): the reference transposes the frontend's (B, 80, frames) output
right after it (train.py:475).
"""
import numpy as np

N_FFT, HOP, N_MELS = 400, 160, 80


def hann_periodic(n=N_FFT):
    k = np.arange(n, dtype=np.float64)
    return 0.5 - 0.5 * np.cos(2.0 * np.pi * k / n)


def _hz_to_mel(f):
    return 2595.0 * np.log10(1.0 + np.asarray(f, np.float64) / 700.0)


def _mel_to_hz(m):
    return 700.0 * (10.0 ** (np.asarray(m, np.float64) / 2595.0) - 1.0)


def melscale_fbanks(sample_rate=16000, n_freqs=N_FFT // 2 + 1, n_mels=N_MELS, f_min=0.0,
                    f_max=None):
    """[n_freqs, n_mels] triangular filterbank (HTK mel, no area normalisation)."""
    f_max = sample_rate / 2.0 if f_max is None else f_max
    all_freqs = np.linspace(0.0, sample_rate / 2.0, n_freqs)
    m_pts = np.linspace(_hz_to_mel(f_min), _hz_to_mel(f_max), n_mels + 2)
    f_pts = _mel_to_hz(m_pts)
    f_diff = f_pts[1:] - f_pts[:-1]
    slopes = f_pts[None, :] - all_freqs[:, None]
    down = -slopes[:, :-2] / f_diff[:-1]
    up = slopes[:, 2:] / f_diff[1:]
    return np.maximum(0.0, np.minimum(down, up))


def dct_ortho(n_mfcc=N_MELS, n_mels=N_MELS):
    """[n_mels, n_mfcc] DCT-II matrix, orthonormal (create_dct(..., norm="ortho"))."""
    n = np.arange(n_mels, dtype=np.float64)
    k = np.arange(n_mfcc, dtype=np.float64)[:, None]
    dct = np.cos(np.pi / n_mels * (n + 0.5) * k)
    dct[0] *= 1.0 / np.sqrt(2.0)
    dct *= np.sqrt(2.0 / n_mels)
    return dct.T


def power_spectrogram(audio):
    """audio [B, N] -> power [B, frames, 201] (center=False)."""
    audio = np.asarray(audio, np.float64)
    B, N = audio.shape
    F = 0 if N < N_FFT else 1 + (N - N_FFT) // HOP
    idx = np.arange(F)[:, None] * HOP + np.arange(N_FFT)[None, :]
    frames = audio[:, idx] * hann_periodic()[None, None, :]
    spec = np.fft.rfft(frames, n=N_FFT, axis=-1)
    return spec.real ** 2 + spec.imag ** 2


def frontend(audio, kind="mfcc", sample_rate=16000):
    """make_frontend(kind)(audio).transpose(1, 2): [B, N] samples -> [B, frames, 80]."""
    mel = power_spectrogram(audio) @ melscale_fbanks(sample_rate)
    if kind == "mfcc":
        return np.log(mel + 1e-6) @ dct_ortho()
    if kind == "mel":
        db = 10.0 * np.log10(np.maximum(mel, 1e-10))
        return np.maximum(db, db.max() - 80.0) if db.size else db
    raise ValueError(f"Unsupported frontend: {kind}")
