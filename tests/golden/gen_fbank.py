#!/usr/bin/env python3
"""Golden fixtures for the feature frontend -> tests/golden/fbank.npz.

The reference's frontend is torchaudio's MFCC / MelSpectrogram + AmplitudeToDB
(model.py:250-279); torchaudio is not installed here (and not in requirements.txt), so parity
w.r.t. torchaudio is UNPINNED.  The fixtures come from INDEPENDENT in-container restatements of
the same published algorithms, which pin oracle/fbank.py:

  power, mel   transformers 5.15.0 ``audio_utils.spectrogram`` (window_function("hann",
               periodic), frame_length = fft_length = 400, hop 160, center=False, power 2.0)
               with ``mel_filter_bank(201, 80, 0, 8000, 16000, norm=None, mel_scale="htk")``
  mfcc         log(mel + 1e-6) then ``scipy.fft.dct(type=2, norm="ortho")`` over the mel axis
  logmel_db    transformers ``power_to_db(mel, reference=1.0, min_value=1e-10, db_range=80)``
               over the whole batch (torchaudio's amplitude_to_DB packs dim -3 for 3-D input)

Run here (CPU):  python tests/golden/gen_fbank.py
Stored: audio [B, N] fp32 (cases: a chirp + noise mix, silence, a clipped square wave), and
fp64-computed outputs in the (B, frames, 80) layout train.py:475 produces, as fp32.
"""
import os

import numpy as np
import scipy.fft
from transformers import audio_utils as au

HERE = os.path.dirname(os.path.abspath(__file__))
SR, N_FFT, HOP, N_MELS = 16000, 400, 160, 80


def reference_style(audio):
    win = au.window_function(N_FFT, "hann", periodic=True)
    fb = au.mel_filter_bank(N_FFT // 2 + 1, N_MELS, 0.0, SR / 2, SR, norm=None, mel_scale="htk")
    power, mel = [], []
    for x in audio.astype(np.float64):
        p = au.spectrogram(x, win, frame_length=N_FFT, hop_length=HOP, fft_length=N_FFT,
                           power=2.0, center=False, dtype=np.float64)           # [201, F]
        power.append(p.T)
        mel.append((fb.T @ p).T)                                               # [F, 80]
    power, mel = np.stack(power), np.stack(mel)
    mfcc = scipy.fft.dct(np.log(mel + 1e-6), type=2, norm="ortho", axis=-1)
    db = au.power_to_db(mel, reference=1.0, min_value=1e-10, db_range=80.0)
    return power, mel, mfcc, db


def main():
    rng = np.random.default_rng(11)
    B, N = 3, 8000
    t = np.arange(N) / SR
    a0 = 0.5 * np.sin(2 * np.pi * (200 + 3000 * t) * t) + 0.05 * rng.standard_normal(N)
    a1 = np.zeros(N)
    a2 = np.clip(0.8 * np.sign(np.sin(2 * np.pi * 440 * t)) + 0.01 * rng.standard_normal(N), -0.7, 0.7)
    audio = np.stack([a0, a1, a2]).astype(np.float32)
    power, mel, mfcc, db = reference_style(audio)
    np.savez_compressed(os.path.join(HERE, "fbank.npz"), audio=audio,
                        power=power.astype(np.float32), mel=mel.astype(np.float32),
                        mfcc=mfcc.astype(np.float32), logmel_db=db.astype(np.float32))
    print({k: v.shape for k, v in dict(audio=audio, power=power, mfcc=mfcc).items()})


if __name__ == "__main__":
    main()
